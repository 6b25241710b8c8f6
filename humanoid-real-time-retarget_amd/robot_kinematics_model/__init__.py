"""Drop-in ``robot_kinematics_model`` (reference robot_kinematics_model/__init__.py:8-12)."""
# overlay: modules this drop-in does not replace (retarget.utils, robot_config.NOITOM, the viewers) resolve to a
# reference checkout that comes later on sys.path
from pkgutil import extend_path
__path__ = extend_path(__path__, __name__)

from robot_kinematics_model.base_robot import RobotZeroPose
from robot_kinematics_model.kinematics import cal_forward_kinematics, cal_local_rotation

__all__ = ["RobotZeroPose", "cal_forward_kinematics", "cal_local_rotation"]
# robot_kinematics_model.hu_forward_model.HuForwardModel / base_forward_model.BaseForwardModel are
# imported by module path, as in the reference.
