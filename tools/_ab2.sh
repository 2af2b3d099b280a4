set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "nullspace or graph or gram_only" > gpurun_out/r03_f_tests.log 2>&1 || { tail -30 gpurun_out/r03_f_tests.log; exit 1; }
tail -1 gpurun_out/r03_f_tests.log
timeout -k 10 200 python tools/gram_only_time.py spot 20000 f64 3 && timeout -k 10 200 python tools/gram_only_time.py spot 20000 bf16 3 && timeout -k 10 200 python tools/gram_only_time.py g1_29dof 125000 f64 3 && timeout -k 10 200 python tools/gram_only_time.py g1_29dof 125000 bf16 3
