set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_q_tests.log 2>&1 || { tail -40 gpurun_out/r03_q_tests.log; exit 1; }
tail -1 gpurun_out/r03_q_tests.log
timeout -k 10 120 python tools/quick_time.py g1_29dof 20000 2>&1 | head -4
timeout -k 10 200 python tools/gram_only_time.py g1_29dof 125000 bf16 3 && timeout -k 10 200 python tools/gram_only_time.py g1_29dof 125000 f64 2 && timeout -k 10 200 python tools/gram_only_time.py g1_29dof 125000 f32 2
