# timing variant: k_exec without the rows phases and the row plans (wrong outputs)
PATCHES = [
    ("backend_hip.hip", "const uint32_t nq = (planned + 3) / 4;", "const uint32_t nq = 0;"),
    ("backend_hip.hip", "const uint32_t units = (R > planned || uni(generalRows)) ? (P == 1 ? R : R * P) : 0u;",
     "const uint32_t units = 0u;"),
    ("backend_hip.hip", "const uint32_t nPairs = sumsStaged ? (planned + 1) / 2 : 0u;", "const uint32_t nPairs = 0u;"),
]
