set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
B="python bench.py --mode bdpt --steps 2 --warmup 1 --no-cpu"
S="python bench.py --mode bdpt --steps 1 --warmup 0 --no-cpu --spp 16"
scripts/gpu_run.sh "gputests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bdpt_def:120:$B" "bdpt_genpk:120:TPT_LIB=variants/genpk/libtpt.so $B" \
  "kt_def:120:TPT_BDPT_SERIAL=1 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_def -o run --output-format csv -- $S" \
  "kt_genpk:120:TPT_BDPT_SERIAL=1 TPT_LIB=variants/genpk/libtpt.so rocprofv3 --kernel-trace --stats -d gpurun_out/kt_genpk -o run --output-format csv -- $S"
for f in gpurun_out/bdpt_*.log; do echo $f $(grep -o '"ms_per_step": [0-9.]*' $f); done
