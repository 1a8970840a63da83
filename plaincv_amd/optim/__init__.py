"""Public exports (mirrors optim/__init__.py)."""
from .base import GradientTransformation, OptState, apply_updates
from .factory import get_optimizer

__all__ = ["GradientTransformation", "OptState", "apply_updates", "get_optimizer"]
