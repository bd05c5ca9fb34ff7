#!/bin/bash
# ISA study of one k_deep instantiation at a given commit, all on the CPU:
#   bash tools/isa/kdeep_isa.sh <git-rev | WORKTREE> <K,BPS,MINW[,EOFROW,STATS]> <out.txt>   (EXTRA="-D..." adds defines)
# builds the instantiation from that commit's kernels.hip (device code only, -S), cuts the function
# out of the assembly and runs the static checks of this directory on it:
#   * resources (SGPRs, spills, VGPRs);
#   * sgpr_mustdef.py — SGPR uses some path reaches without a write;
#   * valueflow.py    — the values every SGPR pair that feeds an address may hold, through the spill
#                       slots (v_writelane / v_readlane): a pointer must hold ONE kernel argument;
#   * vmustdef.py     — vector address registers some path reaches without a write;
#   * the node-list loads (nid / ioff / iend) with the exec mask they are issued under.
set -eo pipefail
REV=$1; INST=${2:-4,3,1}; OUT=$3
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
W=$ROOT/.wt/isa_$REV
mkdir -p $W
if [ "$REV" = WORKTREE ]; then
  cp $ROOT/eds-bwt_amd/csrc/kernels.hip $ROOT/eds-bwt_amd/csrc/kernels.h $W/
else
  git -C $ROOT show $REV:eds-bwt_amd/csrc/kernels.hip > $W/kernels.hip
  git -C $ROOT show $REV:eds-bwt_amd/csrc/kernels.h > $W/kernels.h
fi
printf '#include <hip/hip_runtime.h>\n#include <cstdint>\n#include <cstddef>\n#include "kernels.hip"\nvoid* kdeep_inst() { return (void*)&edsbwt::k_deep<%s>; }\n' "$INST" > $W/inst.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only $EXTRA -S -o $W/all.s $W/inst.hip 2>/dev/null
SYM=$(grep -o "^_ZN6edsbwt6k_deepILi${INST%%,*}[A-Za-z0-9_]*:" $W/all.s | head -1 | tr -d :)
L0=$(grep -n "^$SYM:" $W/all.s | cut -d: -f1)
L1=$(awk -v l=$L0 'NR>l && /s_endpgm/ {print NR; exit}' $W/all.s)
sed -n "${L0},${L1}p" $W/all.s > $W/fn.s
{
  echo "# k_deep<$INST> at $REV ${EXTRA:+($EXTRA) }($( [ "$REV" = WORKTREE ] && echo "the working tree" || git -C $ROOT log -1 --format='%h %s' $REV | cut -c1-100))"
  echo "# compiler: $(/opt/rocm/lib/llvm/bin/clang++ --version | head -1)"
  echo "## resources"
  grep -A14 "\.name: *$SYM" $W/all.s | grep -E "sgpr_count|sgpr_spill|vgpr_count|vgpr_spill|private_segment" | sed 's/^ *//'
  echo "instructions: $(grep -cE '^\s+[a-z]' $W/fn.s), v_writelane: $(grep -c v_writelane $W/fn.s), v_readlane: $(grep -c v_readlane $W/fn.s)"
  echo "## SGPR must-def"
  python3 $ROOT/tools/isa/sgpr_mustdef.py $W/fn.s | tail -12
  echo "## address SGPR pairs: values through the spill slots (listed: pairs that may hold more than one value)"
  python3 $ROOT/tools/isa/valueflow.py $W/fn.s 2>&1 | tail -12
  echo "## vector address registers written on every path"
  python3 $ROOT/tools/isa/vmustdef.py $W/fn.s 2>&1 | tail -8
  echo "## the node-list start: loads through nid / ioff / iend (kernel arguments 0x48 / 0x50 / 0x58) and their exec mask"
  python3 $ROOT/tools/isa/valueflow.py $W/fn.s all 2>/dev/null | grep -E "karg\+0x(48|50|58)'" | head -8
} > $OUT
cat $OUT
