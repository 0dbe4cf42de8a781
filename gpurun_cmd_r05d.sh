bash scripts/steps.sh r05d \
 "replicas_lrn|900|python -u scripts/tierc_replicas.py --fixture c3_1m --worlds 2,4,8 --periods 131072,32768 --combines mean@lrN,touched_mean@lrN --out gpurun_out/r05d_tierc_replicas_c3_1m_lrN.json" \
 "replicas_lrn_blk|900|python -u scripts/tierc_replicas.py --fixture c3_1m --worlds 2,4,8 --periods 131072,32768 --no-overlap --combines mean@lrN --out gpurun_out/r05d_tierc_replicas_c3_1m_lrN_blocking.json"
