"""Build rtg/_frame_post (the teleop frame's host round trip with tensor arguments, rtg/_frame_post.cpp) in-tree.

Host-only C++ against torch's headers and libraries (no GPU code); `__graft_entry__.build()` calls it next to the
HIP library's make.  rtg/realtime.py uses the module when it is present and its ctypes path otherwise.
"""
from __future__ import annotations

import os
import subprocess
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "_frame_post.cpp")


def target() -> str:
    return os.path.join(HERE, "_frame_post" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_frame_post(force: bool = False) -> str:
    out = target()
    if not force and os.path.exists(out) and os.path.getmtime(out) >= os.path.getmtime(SRC):
        return out
    import torch
    t = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-shared", "-fPIC", "-std=c++17", "-DTORCH_EXTENSION_NAME=_frame_post",
           "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-I", os.path.join(t, "include"), "-I", os.path.join(t, "include", "torch", "csrc", "api", "include"),
           "-I", sysconfig.get_paths()["include"], SRC, "-L", os.path.join(t, "lib"), "-lc10", "-ltorch_cpu",
           "-ltorch", "-ltorch_python", "-Wl,-rpath," + os.path.join(t, "lib"), "-o", out]
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build_frame_post(force=True))
