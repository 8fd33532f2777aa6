#!/bin/bash
# GPU-box SQ counter passes (instruction mix, wave-cycle split) of the
# headline render kernel and of the C4 wavefront traversal kernels.
# usage: scripts/profile_instmix.sh r01  (writes gpurun_out/profiles_r01/r01_instmix_*.json)
#   INSTMIX_SCENES="headline c4" (default both); INSTMIX_FRAMES=B: the headline
#   in launches of B frames (the bench's timed launches), written as *_headline_bB.json
set -eu
R=${1:-r01}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles_${R}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_WAVE_CYCLES"
P2="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"
P3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32"
FR=${INSTMIX_FRAMES:-1}
for scene in ${INSTMIX_SCENES:-headline c4}; do
  dirs=()
  i=0
  for pass in "$P1" "$P2" "$P3"; do
    i=$((i + 1))
    d=gpurun_out/instmix_${R}_${scene}_$i
    if [ "$scene" = c4 ]; then
      PMC_SCENE=spheres10k PMC_SIZE=960,540,16 timeout -s KILL 90 rocprofv3 --pmc $pass -d $d -o run --output-format csv \
        -- python3 scripts/pmc_workload.py 2
    else
      PMC_FRAMES=$FR timeout -s KILL 90 rocprofv3 --pmc $pass -d $d -o run --output-format csv -- python3 scripts/pmc_workload.py $([ $FR = 1 ] && echo 5 || echo 2)
    fi
    dirs+=("$d")
  done
  if [ "$scene" = c4 ]; then
    for k in "wf_extend<false, true>" "wf_occlude4<false, true>" "wf_occlude4<false, false>" \
      "wf_cone4<false>" "wf_listtest<false>"; do
      tag=$(echo "$k" | tr -dc 'a-z_,' | tr ',' '_')
      python3 scripts/pmc_instmix.py "$k" gpurun_out/profiles_${R}/${R}_instmix_c4_${tag}.json "${dirs[@]}"
    done
  else
    suf=$([ $FR = 1 ] && echo "" || echo "_b$FR")
    python3 scripts/pmc_instmix.py "render_kernel<false, true, false, false>" gpurun_out/profiles_${R}/${R}_instmix_headline${suf}.json "${dirs[@]}"
  fi
done
echo "instmix ${R} done"
