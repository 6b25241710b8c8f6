"""VTRDYN joint order (retarget/robot_config/VTRDYN.py; identical to the zero-pose asset 'vtrdyn')."""

VTRDYN_JOINT_NAMES = [
    'Hips',
    'RightUpperLeg',
    'RightLowerLeg',
    'RightFoot',
    'LeftUpperLeg',
    'LeftLowerLeg',
    'LeftFoot',
    'Spine',
    'Spine1',
    'Spine2',
    'Spine3',
    'Neck',
    'Head',
    'RightShoulder',
    'RightUpperArm',
    'RightLowerArm',
    'RightHand',
    'LeftShoulder',
    'LeftUpperArm',
    'LeftLowerArm',
    'LeftHand',
]

# parent-indexed topology, connections and graph (VTRDYN.py:33-48), derived from the shipped 21-joint zero pose
# (the 'vtrdyn' asset has exactly these parents) rather than restated
import networkx as nx  # noqa: E402

from rtg import assets as _assets  # noqa: E402

vtrdyn_parent_indices = [int(p) for p in _assets.parents("vtrdyn")]
VTRDYN_CONNECTIONS = [(p, j) for j, p in enumerate(vtrdyn_parent_indices) if p >= 0]
vtrdyn_graph = nx.DiGraph()
for _i, _c in enumerate(VTRDYN_CONNECTIONS):
    vtrdyn_graph.add_node(_i, label=_c)
vtrdyn_graph.add_edges_from(VTRDYN_CONNECTIONS)

from retarget.robot_config import fill_from_checkout  # noqa: E402

fill_from_checkout(globals())
