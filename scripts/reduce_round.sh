#!/usr/bin/env bash
# In the container, after scripts/profile_round.sh TAG pt bdpt c5 pti and
# scripts/gpu_bench_round.sh TAG ran on the GPU box: reduce gpurun_out (or DIR) into the
# committed evidence -- profiles/TAG_{w}_kernel_stats.csv, profiles/TAG_{w}_pmc.txt,
# profiles/TAG_valu_cost.jsonl, profiles/TAG_bench_kernel_stats.csv, the bench line
# appended to profiles/r02_bench_lines.jsonl, and the valu_model.json / traffic.json
# entries bench.py prices its roofline from.
#   scripts/reduce_round.sh TAG BUILD [DIR]
set -eu
tag=$1; build=$2; src=${3:-gpurun_out}
cd "$(dirname "$0")/.."
p=$src/prof_$tag
cp "$p/valu_cost.log" "profiles/${tag}_valu_cost.jsonl"
declare -A desc=([pt]="standard PT 1024 spp, --warmup 1 --steps 1 (2 frames)"
                 [bdpt]="standard BDPT 32 spp, 1 frame" [c5]="bunny BDPT 32 spp, 1 frame"
                 [pti]="standard PT-indirect 64 spp, 1 frame"
                 [c4_ball]="refractive ball PT 1024 spp, 1 frame" [c4_smooth]="smooth dielectric PT 1024 spp, 1 frame")
for w in pt bdpt c5 pti c4_ball c4_smooth; do
  [ -d "$p/${w}_kt" ] || continue
  cp "$p/${w}_kt/run_kernel_stats.csv" "profiles/${tag}_${w}_kernel_stats.csv"
  { echo "# rocprofv3 PMC, $w workload = ${desc[$w]} (scripts/profile_round.sh $tag, build $build); separate passes valu1 / valu2 / misc / fetch / write / lane; values summed over the run's dispatches"
    for pass in valu1 valu2 misc fetch write lane; do
      [ -f "$p/${w}_${pass}/run_counter_collection.csv" ] || continue
      python3 scripts/pmc_summary.py "$p/${w}_${pass}/run_counter_collection.csv"
    done
    if [ -f "$p/${w}_lane/run_counter_collection.csv" ]; then
      echo "# lane utilisation (SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU)) per kernel:"
      python3 scripts/pmc_db.py "$p/${w}_lane/run_counter_collection.csv" | grep -E "^ [a-z_]|lane util"
    fi; } > "profiles/${tag}_${w}_pmc.txt"
done
src_of() { echo "profiles/${tag}_$1_pmc.txt, profiles/${tag}_valu_cost.jsonl"; }
if [ -d "$p/pt_kt" ]; then
  python3 scripts/valu_model.py "$p" standard/pt pt tpt_pt_kernel --frames 2 --samples 629407744 \
      --note "build $build" --source "$(src_of pt)" > /dev/null
  python3 scripts/pmc_traffic.py standard/pt tpt_pt_kernel "$p/pt_fetch/run_counter_collection.csv" \
      "$p/pt_write/run_counter_collection.csv" --frames 2 --note "build $build (profiles/${tag}_pt_pmc.txt)" > /dev/null
fi
if [ -d "$p/bdpt_kt" ]; then
  python3 scripts/valu_model.py "$p" standard/bdpt bdpt tpt_bdpt_ --scale 8 --samples 157351936 \
      --note "build $build; 32-spp profile scaled to the 256-spp frame" --source "$(src_of bdpt)" > /dev/null
  python3 scripts/pmc_traffic.py standard/bdpt tpt_bdpt_ "$p/bdpt_fetch/run_counter_collection.csv" \
      "$p/bdpt_write/run_counter_collection.csv" --frames 0.125 --note "build $build, 32-spp profile x 8 (profiles/${tag}_bdpt_pmc.txt)" > /dev/null
fi
if [ -d "$p/c5_kt" ]; then
  python3 scripts/valu_model.py "$p" bunny/bdpt c5 tpt_bdpt_ --scale 128 --samples 2517630976 \
      --note "build $build; 32-spp profile scaled to the 4096-spp frame" --source "$(src_of c5)" > /dev/null
  python3 scripts/pmc_traffic.py bunny/bdpt tpt_bdpt_ "$p/c5_fetch/run_counter_collection.csv" \
      "$p/c5_write/run_counter_collection.csv" --frames 0.0078125 --note "build $build, 32-spp profile x 128 (profiles/${tag}_c5_pmc.txt)" > /dev/null
fi
if [ -d "$p/pti_kt" ]; then
  python3 scripts/valu_model.py "$p" standard/pti pti tpt_pti_kernel --scale 16 --samples 629407744 \
      --note "build $build; 64-spp profile scaled to the 1024-spp frame" --source "$(src_of pti)" > /dev/null
  python3 scripts/pmc_traffic.py standard/pti tpt_pti_kernel "$p/pti_fetch/run_counter_collection.csv" \
      "$p/pti_write/run_counter_collection.csv" --frames 0.0625 --note "build $build, 64-spp profile x 16 (profiles/${tag}_pti_pmc.txt)" > /dev/null
fi
for c in ball:refractive_ball smooth:smooth_dielectric; do
  w=c4_${c%%:*}; scene=${c#*:}
  if [ -d "$p/${w}_kt" ]; then
    python3 scripts/valu_model.py "$p" $scene/pt $w tpt_pt_kernel --scale 4 --samples 2517630976 \
        --note "build $build; 1024-spp profile scaled to the 4096-spp frame" --source "$(src_of $w)" > /dev/null
    python3 scripts/pmc_traffic.py $scene/pt tpt_pt_kernel "$p/${w}_fetch/run_counter_collection.csv" \
        "$p/${w}_write/run_counter_collection.csv" --frames 0.25 --note "build $build, 1024-spp profile x 4 (profiles/${tag}_${w}_pmc.txt)" > /dev/null
  fi
done
if [ -f "$src/benchkt_$tag/run_kernel_stats.csv" ]; then
  cp "$src/benchkt_$tag/run_kernel_stats.csv" "profiles/${tag}_bench_kernel_stats.csv"
fi
if [ -f "$src/bench_$tag.log" ]; then
  tail -1 "$src/bench_$tag.log" >> "profiles/${tag:0:3}_bench_lines.jsonl"
fi
echo "reduced $p into profiles/${tag}_*"
