"""Drop-in ``poselib.poselib.core.backend`` (reference poselib/poselib/core/backend/__init__.py)."""
from .abstract import Serializable  # noqa: F401
from .logger import logger  # noqa: F401
