set -o pipefail
export TMPDIR=/tmp
for lib in system_identification_amd/libsysid.so tools/_libs/cmp_nolu.so tools/_libs/cmp_noz.so tools/_libs/cmp_none.so; do
  echo "== $lib"
  SYSID_LIB=$PWD/$lib timeout -k 10 120 python tools/gram_only_time.py spot 20000 f64 3 || exit 1
done
bash tools/pmc_cmd.sh gpurun_out/r03_e/g1_f64_full timeout -k 5 100 python tools/k1_only.py g1_29dof 20000 || exit 1
bash tools/pmc_cmd.sh gpurun_out/r03_e/g1_bf16_proj timeout -k 5 100 python tools/k1_gram_only.py g1_29dof 125000 bf16 projector || exit 1
