#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r04g}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kde.py tests/test_gpu_batch.py tests/test_gpu_ties.py tests/test_gpu_dist.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
HOST_PATH_AB=HBX_RESCUE_PASS=1 timeout -k 10 300 python -u tools/host_path.py > $O/host_path.json 2> $O/host_path.err || { tail -20 $O/host_path.err; exit 2; }
python -c "
import json;d=json.load(open('$O/host_path.json'))
for k,v in d.items(): print(k, {a:round(b,1) for a,b in v.items()})"
