# timing variant: every table / window descriptor read from LDS (no memory
# fallback, so no join waits on outstanding loads); wrong for batches whose
# block exceeds the LDS table (the headline's fit)
PATCHES = [
    ("backend_hip.hip", "    return j < kRowsTableLds ? tableL[j] : ld16((uint64_t)(seg + blockWord + i));",
     "    return tableL[j & (kRowsTableLds - 1)];"),
    ("backend_hip.hip", "    return j < kRowsTableLds - kRowSums ? tableL[kRowSums + j] : ld16((uint64_t)(seg + blockWord + kRowSums + e));",
     "    return tableL[(kRowSums + j) & (kRowsTableLds - 1)];"),
]
