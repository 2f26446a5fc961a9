cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_dec1.log 2>&1 || { tail -30 gpurun_out/gpu_tests_dec1.log; exit 1; }
tail -2 gpurun_out/gpu_tests_dec1.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-side > gpurun_out/bench_dec1.log 2>&1 || exit 1
tail -1 gpurun_out/bench_dec1.log | cut -c1-900
timeout -k 10 200 python -u tools/phase_profile.py 20000 > gpurun_out/phase_dec1.log 2>&1 || exit 1
tail -48 gpurun_out/phase_dec1.log
