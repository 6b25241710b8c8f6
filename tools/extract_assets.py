"""Convert the reference's pickled zero poses into plain ``.npz`` assets.

Runs only in the build container (``/root/reference`` is read-only input).
The pickles are decoded by ``rtg.safe_pickle`` (an opcode walker that executes
nothing from the file), never by ``pickle.load``.

Output: ``humanoid-real-time-retarget_amd/assets/<name>.npz`` with
``node_names``, ``parent_indices``, ``local_translation``, ``quat``, ``tensor``,
``is_local``.  Source files:
  hu_v5        <- asset/hu_pose/hu_v5_zero_pose.pkl         (Hu v5 humanoid, 31 links)
  vtrdyn_full  <- asset/zero_pose/vtrdyn_full_zero_pose.pkl (VTRDyn full body+hands, 59)
  vtrdyn       <- asset/zero_pose/vtrdyn_zero_pose.pkl      (VTRDyn body, 21)
  noitom       <- asset/zero_pose/noitom_zero_pose.pkl      (Noitom body, 21)
  hu           <- asset/zero_pose/hu_zero_pose.pkl          (Hu, 33 links / 32 DOFs: HuForwardModel, robot_config/Hu.py)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(HERE), "humanoid-real-time-retarget_amd")
sys.path.insert(0, PKG)

from rtg.safe_pickle import load_skeleton_state_arrays  # noqa: E402

REF = os.environ.get("RTG_REFERENCE", "/root/reference")
ASSETS = {
    "hu_v5": "asset/hu_pose/hu_v5_zero_pose.pkl",
    "vtrdyn_full": "asset/zero_pose/vtrdyn_full_zero_pose.pkl",
    "vtrdyn": "asset/zero_pose/vtrdyn_zero_pose.pkl",
    "noitom": "asset/zero_pose/noitom_zero_pose.pkl",
    "hu": "asset/zero_pose/hu_zero_pose.pkl",
}


def main() -> None:
    out_dir = os.path.join(PKG, "assets")
    os.makedirs(out_dir, exist_ok=True)
    for name, rel in ASSETS.items():
        d = load_skeleton_state_arrays(os.path.join(REF, rel))
        np.savez(
            os.path.join(out_dir, f"{name}.npz"),
            node_names=np.array(d["node_names"]),
            parent_indices=d["parent_indices"],
            local_translation=d["local_translation"],
            quat=d["quat"],
            tensor=d["tensor"],
            is_local=np.array(d["is_local"]),
        )
        print(f"{name}: J={len(d['node_names'])} -> {out_dir}/{name}.npz")


if __name__ == "__main__":
    main()
