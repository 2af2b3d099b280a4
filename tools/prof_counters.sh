#!/bin/bash
# Counter session: kernel times (Spot/G1 20k), K1 SQ counters, K2 SQ counters (Spot, G1), K1 phase stamps.
# Usage: bash tools/prof_counters.sh <tag>      (libsysid.so and libsysid_stamps.so built beforehand)
set -o pipefail
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
L=system_identification_amd/libsysid.so
timeout -k 10 120 python tools/quick_time.py spot 20000 > $OUT/time_spot.txt 2>&1 || { tail $OUT/time_spot.txt; exit 1; }
timeout -k 10 120 python tools/quick_time.py g1_29dof 20000 > $OUT/time_g1.txt 2>&1 || { tail $OUT/time_g1.txt; exit 1; }
bash tools/pmc_k1.sh $L $OUT/k1_spot spot || { echo k1 pmc failed; exit 1; }
bash tools/pmc_k2.sh $L $OUT/k2_spot spot 20000 || { echo k2 spot pmc failed; exit 1; }
bash tools/pmc_k2.sh $L $OUT/k2_g1 g1_29dof 20000 || { echo k2 g1 pmc failed; exit 1; }
python tools/pmc_table.py $OUT/k1_spot/a $OUT/k1_spot/b > $OUT/k1_spot_pmc.txt
python tools/pmc_table.py $OUT/k2_spot/a $OUT/k2_spot/b > $OUT/k2_spot_pmc.txt
python tools/pmc_table.py $OUT/k2_g1/a $OUT/k2_g1/b > $OUT/k2_g1_pmc.txt
if [ -f system_identification_amd/libsysid_stamps.so ]; then
  timeout -k 10 120 python tools/diag_stamps.py spot 20000 > $OUT/stamps_spot.txt 2>&1 || { tail $OUT/stamps_spot.txt; exit 1; }
fi
cat $OUT/time_spot.txt $OUT/time_g1.txt
echo DONE
