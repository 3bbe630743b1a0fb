set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
# Bunny scene (BASELINE config 5): flat queries with the bunny mesh as a walk group
# (default) vs threaded walks everywhere (TPT_FLAT=0), plus the Standard headline lines.
T="python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread"
scripts/gpu_run.sh "t_gpu:400:$T" \
  "bun_pt:120:python bench.py --scene bunny --mode pt --steps 2 --warmup 1 --no-cpu" \
  "bun_pt_walk:120:TPT_FLAT=0 python bench.py --scene bunny --mode pt --steps 2 --warmup 1 --no-cpu" \
  "bun_bdpt:180:python bench.py --scene bunny --mode bdpt --steps 1 --warmup 1 --no-cpu" \
  "bun_bdpt_walk:180:TPT_FLAT=0 python bench.py --scene bunny --mode bdpt --steps 1 --warmup 1 --no-cpu" \
  "std_pt:120:python bench.py --mode pt --steps 3 --warmup 1 --no-cpu" \
  "std_bdpt:120:python bench.py --mode bdpt --steps 2 --warmup 1 --no-cpu"
for f in gpurun_out/bun_*.log gpurun_out/std_*.log; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $f); done
