"""GPU sampler timing at 1e6 x 32 (bench side line gpu_sampler): python tools/time_sampler2.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from hpbandster_amd import kde  # noqa: E402
from hpbandster_amd import synthetic as S  # noqa: E402

dev = torch.device("cuda", 0)
X = S.make_observations(10000, 24, 8, 4)
L = S.make_losses(10000)
pair = kde.fit_pair(X, L, S.var_type_string(24, 8), 33, device=dev)
ws = torch.empty(pair.workspace_bytes(1000000), dtype=torch.uint8, device=dev)
print(bench.sampler_line(pair, dev, 24, 8, 4, 1000000, ws))
