"""poselib mirror: ``poselib.poselib.core.rotation3d`` and ``poselib.poselib.skeleton.skeleton3d``
(reference poselib/poselib/__init__.py) with all arithmetic on the MI355X."""
__version__ = "0.0.1"

from .core import *  # noqa: F401,F403
