# variant: descriptor reads past the LDS table wait for their own load inside
# the fallback branch (vmcnt(0) there), so the common LDS path joins with no
# pending memory load and no wait on unrelated outstanding loads
PATCHES = [
    ("backend_hip.hip", "    return j < kRowsTableLds ? tableL[j] : ld16((uint64_t)(seg + blockWord + i));",
     "    if (j < kRowsTableLds)\n        return tableL[j];\n    const uint4 v = ld16((uint64_t)(seg + blockWord + i));\n    __builtin_amdgcn_s_waitcnt(0x0F70);\n    return v;"),
    ("backend_hip.hip", "    return j < kRowsTableLds - kRowSums ? tableL[kRowSums + j] : ld16((uint64_t)(seg + blockWord + kRowSums + e));",
     "    if (j < kRowsTableLds - kRowSums)\n        return tableL[kRowSums + j];\n    const uint4 v = ld16((uint64_t)(seg + blockWord + kRowSums + e));\n    __builtin_amdgcn_s_waitcnt(0x0F70);\n    return v;"),
]
