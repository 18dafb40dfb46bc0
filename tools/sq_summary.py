"""Per-kernel SQ counter summary of tools/sq_profile.sh output."""
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float))
for row in csv.DictReader(open(sys.argv[1])):
    name = row["Kernel_Name"].split("(")[0].replace("void ", "")
    acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
for k, c in acc.items():
    if not k.startswith("k_"):
        continue
    wc = c["SQ_WAVE_CYCLES"] or 1
    print(f"{k:26s} wait_any {c['SQ_WAIT_ANY']/wc:5.2f} wait_inst {c['SQ_WAIT_INST_ANY']/wc:5.2f} "
          f"active {c['SQ_ACTIVE_INST_ANY']/wc:5.2f}  valu_insts {c['SQ_INSTS_VALU']:.3e} vmem_rd {c['SQ_INSTS_VMEM_RD']:.3e} "
          f"valu_util {c['SQ_THREAD_CYCLES_VALU']/max(64*c['SQ_ACTIVE_INST_VALU'],1):5.2f}")
