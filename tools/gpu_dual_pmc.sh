#!/bin/bash
# PMC passes on the dual-kite kernel (one rocprofv3 run per counter group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIB=${LIB:-}
i=0
IFS=';' read -ra G <<< "${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD;SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY}"
for grp in "${G[@]}"; do
  i=$((i+1))
  echo "=== pmc group $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/dpmc$i -o run --output-format csv -- python tools/dual_prof.py --iters 3 $LIB > gpurun_out/dual_pmc$i.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -2 gpurun_out/dual_pmc$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo ALL_DONE
