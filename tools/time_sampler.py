"""ms per hbx_kde_sample launch (1e6 x 32 candidates around config #3's good KDE); the library is
HBX_LIB_PATH's (ablation builds) or the regular one."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpbandster_amd import kde  # noqa: E402
from hpbandster_amd import synthetic as S  # noqa: E402

dev = torch.device("cuda", 0)
X = S.make_observations(10000, 24, 8, 4)
pair = kde.fit_pair(X, S.make_losses(10000), S.var_type_string(24, 8), 33, device=dev)
lv = np.array([0] * 24 + [4] * 8)
for table in (True, False):
    pair.good.sample(lv, 3.0, 1000000, seed=1, counter_base=0, table=table)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(10):
        pair.good.sample(lv, 3.0, 1000000, seed=1, counter_base=k, table=table)
    e1.record()
    torch.cuda.synchronize()
    print("%s table=%s: %.3f ms" % (os.environ.get("HBX_LIB_PATH", "regular"), table, e0.elapsed_time(e1) / 10))
