#!/usr/bin/env python3
"""Register/LDS/spill summary of the rt580 kernels from the device assembly
(make -C 580-raytracer_amd asm). Usage: tools/kernel_regs.py [name-filter]"""
import os
import re
import sys

import yaml

path = os.path.join(os.path.dirname(__file__), "..", "580-raytracer_amd", "_build", "rt_kernels.s")
text = open(path).read()
meta = text[text.index("amdhsa.kernels:"):]
meta = meta[:meta.index(".end_amdgpu_metadata")]
meta = "\n".join(l for l in meta.splitlines() if l.strip() and not l.startswith("\t"))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for k in yaml.safe_load(meta)["amdhsa.kernels"]:
    name = k[".name"]
    if "rt580" not in name or flt not in name:
        continue
    short = re.sub(r"^_ZN5rt580\d+", "", name)[:60]
    print("%-60s vgpr %3d sgpr %3d spill v%d s%d scratch %d lds %d" % (
        short, k[".vgpr_count"], k[".sgpr_count"], k.get(".vgpr_spill_count", 0), k.get(".sgpr_spill_count", 0),
        k[".private_segment_fixed_size"], k[".group_segment_fixed_size"]))
