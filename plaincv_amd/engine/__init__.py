"""Engine API (mirrors engine/__init__.py + engine/flax_engine.py)."""
from .engine import (GraphedTrainStep, TrainState, compute_metrics, create_train_state, cross_entropy_loss,
                     make_eval_step, make_train_step)

__all__ = ["TrainState", "create_train_state", "make_train_step", "make_eval_step", "cross_entropy_loss",
           "compute_metrics", "GraphedTrainStep"]
