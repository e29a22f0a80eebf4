#!/bin/bash
# SQ counters of K4 alone (tools/exp_varint.cpp, uniform int64 shares), two passes of 8 SQ counters
# each (one block per pass, as the guide's PMC section prescribes).  Out: gpurun_out/${TAG:-pmcv}/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${TAG:-pmcv}
mkdir -p "$out"
p1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES"
p2="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA"
i=1
for pass in "$p1" "$p2"; do
    timeout -s KILL 60 rocprofv3 --pmc $pass -d "$out/pass$i" -o run --output-format csv -- \
        tools/_exp_varint 11689512 5 0 > "$out/pass$i.log" 2>&1 || { tail -20 "$out/pass$i.log"; exit 1; }
    i=$((i + 1))
done
python3 tools/pmc_table.py "$out"
