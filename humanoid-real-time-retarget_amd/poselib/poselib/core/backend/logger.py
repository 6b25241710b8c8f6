"""The ``poselib`` logger (reference poselib/poselib/core/backend/logger.py:10-20)."""
import logging

logger = logging.getLogger("poselib")
logger.setLevel(logging.INFO)
if not logger.handlers:
    _h = logging.StreamHandler()
    _h.setFormatter(logging.Formatter(fmt="%(asctime)-15s - %(levelname)s - %(module)s - %(message)s"))
    logger.addHandler(_h)
