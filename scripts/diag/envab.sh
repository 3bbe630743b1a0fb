cd $GRAFT_REPO_ROOT
scripts/ab_variants.sh "--mode bdpt --steps 3 --warmup 1" ABL_NOK1 ABL_NOQ
for f in 2 1 0; do echo "TPT_FLAT=$f $(TPT_FLAT=$f timeout -k 10 120 python bench.py --mode bdpt --steps 3 --warmup 1 --no-cpu 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')" | tee -a gpurun_out/ab.log; done
