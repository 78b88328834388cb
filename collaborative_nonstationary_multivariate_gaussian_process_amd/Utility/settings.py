"""code/SIM_code/Utility/settings.py."""
import torch

jitter = 1e-6
torchType = torch.DoubleTensor
precision = 1e-6
