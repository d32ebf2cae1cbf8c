#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-r04o}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 2; }
python3 -c "
import json;b=json.loads(open('$O/bench.json').read().strip().split('\n')[-1]);print(b['value'], b['roofline']['frac']); print({k:(b[k].get('ms_sequential'),b[k].get('ms_batched'),b[k].get('speedup')) for k in ('sh_stage','sh_stage_interleaved','sh_stage_interleaved_host_sampler')})"
