# round-6 final-tree evidence in one call: the whole -m gpu suite, the default bench, smoke()
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests \
  > gpurun_out/r06_gputests_final.log 2>&1 || { tail -30 gpurun_out/r06_gputests_final.log; exit 1; }
tail -2 gpurun_out/r06_gputests_final.log
timeout -k 10 600 python3 bench.py > gpurun_out/r06_bench_final.log 2>&1 || { tail -20 gpurun_out/r06_bench_final.log; exit 1; }
grep '^{' gpurun_out/r06_bench_final.log | tail -1 > gpurun_out/r06_bench_final.json
cut -c1-300 gpurun_out/r06_bench_final.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
echo callC-ok
