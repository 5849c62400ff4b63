#!/usr/bin/env python3
"""Issue rate of the kNN insertion's compares against the v_fma_f32 peak (fbr_valu_peak kinds 3 / 4):
is a 64-bit unsigned compare one VALU issue slot, like a 32-bit one?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from feature_base_pointcloud_registration_amd import api  # noqa: E402

for kind, name in ((0, "v_fma_f32"), (3, "v_cmp_lt_u64"), (4, "v_cmp_lt_u32")):
    for w in (4, 8):
        g, ms = api.valu_peak(0, w, kind, 4096, 5)
        print(f"{name:14s} waves/SIMD {w}: {g:8.1f} G wave-instr/s ({ms:.3f} ms per launch)")
