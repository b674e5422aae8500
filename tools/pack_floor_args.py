#!/usr/bin/env python3
"""Arguments for tools/pack_floor_probe: NAME SPAN PACKED per CFG-C type at
the given packed size (count = packed // size instances; span = extent *
(count - 1) + true_ub - true_lb, the bytes a pack reads)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import golden_io  # noqa: E402

TYPES = ["vector_f32_b1_s2", "vector_f32_b4_s8", "vector_f64_b3_s5", "vector_f32_b16_s32", "vector_f32_b64_s128",
         "indexed_f32_random", "struct_char_d3_int_resized48", "ref_blacs_indexed", "ref_struct", "ref_strange"]
packed = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
_, recs = golden_io.ddt_records()
out = []
for name in TYPES:
    r = next(x for x in recs if x["name"] == name)
    count = packed // r["size"]
    span = (r["ub"] - r["lb"]) * (count - 1) + r["true_ub"] - r["true_lb"]
    out += [name, str(span), str(count * r["size"])]
print(" ".join(out))
