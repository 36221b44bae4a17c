#!/bin/bash
# Clock and MFMA-busy of the search kernel for library variants (build/variants/<name>.so): one rocprofv3 PMC
# pass each over tools/run_search.py. usage: tools/pmc_clock.sh name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for v in "$@"; do
  OUT=gpurun_out/clk_$v
  CRIMP_LIB=build/variants/$v.so timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d "$OUT" -o pmc --output-format csv -- python3 tools/run_search.py > "$OUT.log" 2>&1
  rc=$?; echo "[$v] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 tools/pmc_summary.py "$OUT" k_search_exact > "$OUT/summary.txt"
  python3 - "$OUT/summary.txt" <<'PY'
import sys, re
d = {}
for l in open(sys.argv[1]):
    p = l.split()
    if len(p) == 2: d[p[0]] = float(p[1])
    if l.startswith("kernel ns"): ns = sum(eval(l.split(":", 1)[1]))
clk = d["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9)
simd_cyc = 1024 * clk * ns * 1e-9
print("  kernel %.1f ms  clock %.3f GHz  MFMA busy %.1f %%  VALU/MFMA %.2f  wait_any %.1f %%  wait_inst %.1f %% of wave cycles" % (
    ns / 1e6, clk / 1e9, 100 * d["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cyc, d["SQ_INSTS_VALU"] / d["SQ_INSTS_MFMA"],
    100 * d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"], 100 * d["SQ_WAIT_INST_ANY"] / d["SQ_WAVE_CYCLES"]))
PY
done
