# variant: the lane-mode update partials folded across the wave's halves
# (one v_permlane32_swap + XOR per dword) before the LDS XOR atomics, which
# then come from two quads (2-way bank conflicts instead of 4-way)
PATCHES = [
    ("backend_hip.hip", "                                    // (the quads hold different elements: each adds its share)\n                                    if (la) {",
     """                                    {
                                        auto f32 = [](uint32_t v) {
                                            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
                                            return r[0] ^ r[1];
                                        };
                                        A0 = make_uint4(f32(A0.x), f32(A0.y), f32(A0.z), f32(A0.w));
                                        A1 = make_uint4(f32(A1.x), f32(A1.y), f32(A1.z), f32(A1.w));
                                        A2 = make_uint4(f32(A2.x), f32(A2.y), f32(A2.z), f32(A2.w));
                                    }
                                    if (la && lane < 32) {"""),
    ("backend_hip.hip", "                                    if (lb) {\n                                        atomicXor(&updAcc[ub * 64 + b4 + 0], A1.x);",
     "                                    if (lb && lane < 32) {\n                                        atomicXor(&updAcc[ub * 64 + b4 + 0], A1.x);"),
    ("backend_hip.hip", "                                    if (lc) {\n                                        atomicXor(&updAcc[uc * 64 + b4 + 0], A2.x);",
     "                                    if (lc && lane < 32) {\n                                        atomicXor(&updAcc[uc * 64 + b4 + 0], A2.x);"),
]
