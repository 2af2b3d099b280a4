set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "reduced or config5 or gram_only or bf16" > gpurun_out/r03_q_tests.log 2>&1 || { tail -40 gpurun_out/r03_q_tests.log; exit 1; }
grep -i "bf16\|passed\|failed" gpurun_out/r03_q_tests.log | tail -20
timeout -k 10 200 python tools/gram_only_time.py g1_29dof 125000 bf16 3 && timeout -k 10 200 python tools/gram_only_time.py spot 20000 bf16 3
