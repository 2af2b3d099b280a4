#!/bin/bash
# Round-4 session 3: why the streamed inputs' flags do not land while K1 runs (stream-flag micro test, HW queue count,
# flag by WriteValue32, a kernel + memory-copy trace of the streamed call), then the record's rocprofv3 stats and
# FETCH/WRITE + SQ counter passes (tools/gpu_r04_final_b.sh).
set -o pipefail
TAG=${1:-r04_s3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench/stream_flag 1 > $OUT/stream_flag_1.txt 2>&1; echo "stream_flag 1 rc $?"; cat $OUT/stream_flag_1.txt
timeout -k 10 60 ./tools/ubench/stream_flag 2048 > $OUT/stream_flag_2048.txt 2>&1; echo "stream_flag 2048 rc $?"; tail -8 $OUT/stream_flag_2048.txt
SYSID_STREAM_PARTS=2 SYSID_TRACE_HOST=1 timeout -k 10 60 python tools/stream_probe.py 3 > $OUT/streamed_default.txt 2>&1 || exit 1; echo "== default"; cat $OUT/streamed_default.txt
GPU_MAX_HW_QUEUES=8 SYSID_STREAM_PARTS=2 SYSID_TRACE_HOST=1 timeout -k 10 60 python tools/stream_probe.py 3 > $OUT/streamed_hwq8.txt 2>&1 || exit 1; echo "== hwq 8"; cat $OUT/streamed_hwq8.txt
SYSID_STREAM_FLAG=write SYSID_STREAM_PARTS=2 SYSID_TRACE_HOST=1 timeout -k 10 60 python tools/stream_probe.py 3 > $OUT/streamed_write.txt 2>&1 || exit 1; echo "== flag write"; cat $OUT/streamed_write.txt
SYSID_STREAM_PARTS=2 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $OUT/trace -o run -- python tools/stream_probe.py 2 > $OUT/trace.log 2>&1 || exit 1
find $OUT/trace -name "*.csv"
bash tools/gpu_r04_final_b.sh $TAG/rec || exit 1
echo S3_DONE
