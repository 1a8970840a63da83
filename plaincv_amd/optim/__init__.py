"""Public exports (mirrors optim/__init__.py)."""
from .base import GradientTransformation, OptState, apply_updates
from .factory import get_optimizer
from .schedule_free import ScheduleFree
from .signum import Signum

__all__ = ["GradientTransformation", "OptState", "ScheduleFree", "Signum", "apply_updates", "get_optimizer"]
