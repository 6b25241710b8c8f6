"""retarget/torch_ext.py:10-21 -- float32 conversion helpers."""
import torch


def to_numpy(tensor):
    return tensor.cpu().numpy() if torch.is_tensor(tensor) else tensor


def to_torch(tensor):
    return tensor if torch.is_tensor(tensor) else torch.from_numpy(tensor).to(torch.float32)
