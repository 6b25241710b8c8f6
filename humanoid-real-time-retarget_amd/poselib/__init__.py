"""Drop-in mirror of the reference's ``poselib`` package (hot-path subset), backed by librtg_hip."""
