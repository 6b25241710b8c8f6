"""Drop-in ``poselib.poselib.core`` (reference poselib/poselib/core/__init__.py:1-3): the same three imports."""
# overlay: modules this drop-in does not replace (retarget.utils, robot_config.NOITOM, the viewers) resolve to a
# reference checkout that comes later on sys.path
from pkgutil import extend_path
__path__ = extend_path(__path__, __name__)

from .tensor_utils import *  # noqa: F401,F403
from .rotation3d import *  # noqa: F401,F403
from .backend import Serializable, logger  # noqa: F401
