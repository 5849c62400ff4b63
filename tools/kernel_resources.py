"""Print VGPR / SGPR / LDS / scratch of every kernel in hipcc -S assembly files.
usage: kernel_resources.py FILE.s [FILE.s ...]"""
import re
import sys

for f in sys.argv[1:]:
    s = open(f).read()
    for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", s, re.S):
        body = m.group(2)

        def g(k):
            r = re.search(r"\.amdhsa_" + k + r" (\d+)", body)
            return r.group(1) if r else "?"

        print(f"{m.group(1)[:72]:72s} vgpr={g('next_free_vgpr'):>4} sgpr={g('next_free_sgpr'):>4} "
              f"lds={g('group_segment_fixed_size'):>6} scratch={g('private_segment_fixed_size')}")
