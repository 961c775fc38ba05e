#!/usr/bin/env python
"""Per-kernel register / scratch summary of a hipcc --cuda-device-only -S
listing (metadata block of each kernel), optionally filtered by a name
fragment: python tools/isa_summary.py /tmp/rows_f32.s k_sgd_strata"""
import re
import sys

text = open(sys.argv[1]).read()
needle = sys.argv[2] if len(sys.argv) > 2 else ""
for blk in re.split(r"\n\s+- \.agpr_count", text)[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or needle not in name.group(1):
        continue
    get = lambda key: (re.search(r"\." + key + r":\s+(\d+)", blk) or [None, "?"])[1]  # noqa: E731
    print(f"{name.group(1)[:90]:90s} vgpr={get('vgpr_count'):>4s} "
          f"scratch={get('private_segment_fixed_size'):>5s} spill={get('vgpr_spill_count')}")
