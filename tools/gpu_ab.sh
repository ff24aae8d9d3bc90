# A/B of abl_libs/*.so on bench kernel times: BARGS (bench args) per config list in CFGS
set -e
mkdir -p gpurun_out
for cfg in ${CFGS:-metric}; do
  BARGS="--config $cfg ${BARGS0}" KFILT=${KFILT:-x} timeout -k 10 600 bash tools/ab_libs.sh
done
