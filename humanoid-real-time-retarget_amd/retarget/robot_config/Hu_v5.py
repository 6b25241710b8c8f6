"""Hu v5 humanoid tables (retarget/robot_config/Hu_v5.py:12-33).

DOF k drives link k+1 about axis Hu_DOF_AXIS[k] (0=x, 1=y, 2=z).  The limit
tables are carried over as data; the reference never applies them on the
retarget path (and they hold 32 entries for 30 DOFs).
"""
import torch

Hu_DOF_AXIS = [
    2, 0, 1, 1, 1,
    2, 0, 1, 1, 1,
    2,
    1, 0, 2, 1, 0, 1, 2, 1, 1,
    1, 0, 2, 1, 0, 1, 2, 1, 1,
    2, ]

Hu_DOF_LOWER = torch.Tensor([
    -0.1745, -0.3491, -1.5708, 0.0997, -0.6981, -0.3665,
    -0.1745, -0.3491, -1.5708, 0.0997, -0.6981, -0.3665,
    -1.0472,
    -3.1416, 0., -1.5708, 0., -1.5708, -0.785, -0.7854, 0., -0.044,
    -3.1416, -1.5708, -1.5708, 0., -1.5708, -0.785, -0.7854, 0., -0.044,
    -1., ])
Hu_DOF_UPPER = torch.Tensor([
    0.1745, 0.3491, 0.8727, 2.618, 0.6981, 0.3665,
    0.1745, 0.3491, 0.8727, 2.618, 0.6981, 0.3665,
    1.0472,
    1.0472, 1.5708, 1.5708, 1.5708, 1.5708, 0.785, 0.7854, 0.044, 0.,
    1.0472, 0., 1.5708, 1.5708, 1.5708, 0.785, 0.7854, 0.044, 0.,
    1., ])

from retarget.robot_config import fill_from_checkout  # noqa: E402

fill_from_checkout(globals())   # the reference's viewer graphs / joint mappings, when a checkout is overlaid
