# timing variant: k_exec without the sum updates and their stores (wrong outputs)
PATCHES = [
    ("backend_hip.hip", "const uint32_t uUnits = U * Q;", "const uint32_t uUnits = 0;"),
    ("backend_hip.hip", "for (uint32_t u = wave; u < U; u += kExecWaves) {", "for (uint32_t u = wave; u < 0u; u += kExecWaves) {"),
]
