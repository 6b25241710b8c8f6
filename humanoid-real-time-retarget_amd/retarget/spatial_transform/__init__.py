# overlay: modules this drop-in does not replace (retarget.utils, robot_config.NOITOM, the viewers) resolve to a
# reference checkout that comes later on sys.path
from pkgutil import extend_path
__path__ = extend_path(__path__, __name__)
