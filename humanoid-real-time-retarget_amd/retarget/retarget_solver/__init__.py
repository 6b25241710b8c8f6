"""Drop-in ``retarget.retarget_solver`` (reference retarget/retarget_solver/__init__.py:9-14)."""
# overlay: modules this drop-in does not replace (retarget.utils, robot_config.NOITOM, the viewers) resolve to a
# reference checkout that comes later on sys.path
from pkgutil import extend_path
__path__ = extend_path(__path__, __name__)

from retarget.retarget_solver.retarget_solver import HuUpperBodyFromMocapRetarget
from retarget.retarget_solver.body_retargeter import Mocap2HuBodyRetargeter
from retarget.retarget_solver.full_body_retargeter import VtrdynFullBodyRetargeter
from retarget.retarget_solver.full_body_pos_retargeter import VtrdynFullBodyPosRetargeter

__all__ = ['HuUpperBodyFromMocapRetarget', 'Mocap2HuBodyRetargeter', 'VtrdynFullBodyRetargeter',
           'VtrdynFullBodyPosRetargeter']
