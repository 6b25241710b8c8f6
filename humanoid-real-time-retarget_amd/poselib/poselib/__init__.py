"""poselib mirror: ``poselib.poselib.core.rotation3d`` and ``poselib.poselib.skeleton.skeleton3d``
(reference poselib/poselib/__init__.py) with all arithmetic on the MI355X."""
# overlay: modules this drop-in does not replace (retarget.utils, robot_config.NOITOM, the viewers) resolve to a
# reference checkout that comes later on sys.path
from pkgutil import extend_path
__path__ = extend_path(__path__, __name__)

__version__ = "0.0.1"

from .core import *  # noqa: F401,F403
