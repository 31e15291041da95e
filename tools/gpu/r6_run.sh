# Round-6 probe: the tuning suite (hook_up branches against the oracle) and the sparse-etree
# tuning A/B (tools/tune_ab.py: one 1/8 shard's map and the 8-tree K-way merge per variant).
set -o pipefail
mkdir -p gpurun_out/r6 && export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_tuning.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r6/tuning_c.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/tune_ab.py 26 5 8 up1:hook_up=1 up1b:hook_up=1,hook_batch=1 up2:hook_up=2 > gpurun_out/r6/tune_ab_hookup.json 2> gpurun_out/r6/tune_ab_hookup.err || exit 1
