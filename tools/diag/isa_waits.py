"""Prints a kernel's vector-memory instructions and s_waitcnt lines in order from the build's ISA listing (make asm),
with the VGPR/spill summary -- to check where the compiler makes a wave wait on which loads/atomics.
Usage: python tools/diag/isa_waits.py <mobheat-gfx950.s> <symbol substring> [context-regex]"""
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
pat = re.compile(sys.argv[3]) if len(sys.argv) > 3 else re.compile(
    r"s_waitcnt|global_load|global_store|global_atomic|buffer_|s_cbranch|^\.LBB|ds_read|ds_write|scratch_|s_barrier")
s = open(path).read()
m = re.search(r"^(" + r"\w*" + re.escape(sym) + r"\w*):", s, re.M)
if not m:
    sys.exit(f"no symbol containing {sym}")
name = m.group(1)
a = m.end()
b = s.index(".Lfunc_end", a)
for i, l in enumerate(s[a:b].split("\n")):
    if pat.search(l):
        print(i, l.strip())
for key in ("num_vgpr", "private_seg_size", "sgpr_spill_count", "vgpr_spill_count"):
    mm = re.search(r"\.set " + re.escape(name) + r"\." + key + r", (.*)", s)
    if mm:
        print(key, mm.group(1))
mm = re.search(r"\.amdhsa_kernel " + re.escape(name) + r"(.*?)\.end_amdhsa_kernel", s, re.S)
if mm:
    for k in ("group_segment_fixed_size", "next_free_vgpr", "private_segment_fixed_size"):
        x = re.search(r"\.amdhsa_" + k + r" (\S+)", mm.group(1))
        if x:
            print(k, x.group(1))
