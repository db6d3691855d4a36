export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k hash_spgemm --timeout 120 --timeout-method thread > gpurun_out/t_hash3.log 2>&1 || exit 1
for g in 100000 2 4 8 16; do
  timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline --steps 4 --spgemm-steps 3 --knob window_in_c_groups=$g > gpurun_out/sweep_$g.log 2>&1 || exit 1
  python -c "import json,sys;d=json.loads(open('gpurun_out/sweep_$g.log').read().strip().splitlines()[-1]);print($g, d['secondary']['config5_spgemm_plus_times_fp64']['ms'])"
done
