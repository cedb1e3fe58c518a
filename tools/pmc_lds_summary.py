"""Per-kernel LDS-array and vector-ALU activity from a tools/pmc_lds.sh pass.

    python tools/pmc_lds_summary.py gpurun_out/<tag>

GRBM_GUI_ACTIVE is summed over the 8 XCDs, so the kernel's busy cycles are GUI/8; per CU the
LDS array was active SQ_LDS_IDX_ACTIVE/256 cycles (bank-conflict cycles SQ_LDS_BANK_CONFLICT/256);
a wave64 VALU instruction occupies a SIMD-32 for 2 cycles (MI355X_MICROARCH.md), so the vector
ALUs were busy SQ_INSTS_VALU*2/1024 cycles per SIMD.
"""
import collections
import csv
import glob
import sys

XCDS, CUS, SIMDS = 8, 256, 1024
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/pmc_lds/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "fsem" in r["Kernel_Name"]:
            acc[r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]][r["Counter_Name"]] += float(r["Counter_Value"])
print(f"{'kernel':40s} {'ms@2.4GHz':>9s} {'LDS array':>9s} {'bank conf':>9s} {'VALU':>6s}")
for k, v in acc.items():
    g = max(v["GRBM_GUI_ACTIVE"] / XCDS, 1.0)
    print(f"{k:40s} {g / 2.4e6:9.3f} {v['SQ_LDS_IDX_ACTIVE'] / CUS / g:9.3f} {v['SQ_LDS_BANK_CONFLICT'] / CUS / g:9.3f} "
          f"{v['SQ_INSTS_VALU'] * 2 / SIMDS / g:6.3f}")
