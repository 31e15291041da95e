# Oracle digests for the full-size configs (tools/make_scale_golden.py), one per call:
#   CFG=c3 bash gpugold.sh   -> gpurun_out/golden/c3.json (+ .log)
set -o pipefail
mkdir -p gpurun_out/golden && export HSA_ENABLE_IPC_MODE_LEGACY=0 && export TMPDIR=/tmp
( while true; do date >> gpurun_out/heartbeat.txt; sleep 50; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 ${LIMIT:-1100} python -u tools/make_scale_golden.py $CFG --threads 16 --out gpurun_out/golden/$CFG.json \
  > gpurun_out/golden/$CFG.out 2> gpurun_out/golden/$CFG.log
