set -o pipefail
mkdir -p gpurun_out/fab
timeout -k 10 180 python -u tools/fwd_check.py > gpurun_out/fab/check.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fab/tests.log 2>&1 || { tail -30 gpurun_out/fab/tests.log; exit 1; }
tail -2 gpurun_out/fab/tests.log
timeout -k 10 120 python -u tools/z2_probe.py > gpurun_out/fab/probe_split.txt 2>&1 && tail -1 gpurun_out/fab/probe_split.txt
# (A/B of round 5: the env switch MEPOL_FWD_FUSED was removed once the split form won)
