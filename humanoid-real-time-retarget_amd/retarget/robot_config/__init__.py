# overlay: modules this drop-in does not replace (retarget.utils, robot_config.NOITOM, the viewers) resolve to a
# reference checkout that comes later on sys.path
from pkgutil import extend_path
__path__ = extend_path(__path__, __name__)


def fill_from_checkout(g: dict) -> bool:
    """The reference's table modules (retarget/robot_config/*.py) also hold viewer graphs and joint mappings that no
    solver reads.  When a reference checkout is overlaid (a later entry of this package's __path__), copy every public
    name of the checkout's same-named module that the drop-in module does not define itself, so callers of the full
    table surface keep working; without a checkout only the drop-in's tables exist."""
    import importlib.util
    import os
    fname = g["__name__"].rsplit(".", 1)[1] + ".py"
    here = os.path.dirname(os.path.abspath(g["__file__"]))
    for d in __path__:
        p = os.path.join(d, fname)
        if os.path.abspath(d) == here or not os.path.exists(p):
            continue
        spec = importlib.util.spec_from_file_location(g["__name__"] + "_checkout", p)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        for k, v in vars(mod).items():
            if not k.startswith("_") and k not in g:
                g[k] = v
        return True
    return False
