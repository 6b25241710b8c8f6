from .rotation3d import *  # noqa: F401,F403
