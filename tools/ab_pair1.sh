set -o pipefail
mkdir -p gpurun_out/ct1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_full_winners.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/ct1/pytest.log 2>&1 || { tail -30 gpurun_out/ct1/pytest.log; exit 1; }
tail -2 gpurun_out/ct1/pytest.log
for i in 1 2 3; do for v in 1 0; do
  env HBX_PAIR1=$v timeout -k 10 200 python -u tools/side_lines.py config2 getconfig > gpurun_out/ct1/sl_${v}_$i.json 2>/dev/null || exit 2
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ct1/sl_${v}_$i.json').read().strip().splitlines()[-1])
c=d['config2']; g=d['get_config_default']
print('PAIR1=$v run $i config2 step %.2f us scoring %.2f us ok %s | get_config %.4f ms best %.4f' % (c['ms_per_step']*1e3, c['scoring_launch_ms']*1e3, c['winner_ok'], g['ms_per_call'], g['ms_per_call_best']))"
done; done
