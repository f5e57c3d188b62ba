# profiling variant: k_exec phase clocks kept in LDS by thread 0 and flushed
# once per workgroup (the in-loop PHASE_ADD atomics dropped), so the
# instrumentation barely perturbs what it measures.  Build with
#   python tools/variant_src.py phase2 tools/variants/exec_phase2.py -DSGPU_PHASE_CLOCKS
PATCHES = [
    ("backend_hip.hip", "            atomicAdd(&g_phaseClk[k], now_ - (t));                                   \\\n",
     "            phL[k] += now_ - (t);                                                    \\\n"),
    ("backend_hip.hip", "        if ((threadIdx.x & 63) == 0)                                                 \\\n            atomicAdd(&g_phaseClk[k], (unsigned long long)(v));                      \\\n",
     "        if (false)                                                                   \\\n            atomicAdd(&g_phaseClk[k], (unsigned long long)(v));                      \\\n"),
    ("backend_hip.hip", "    __shared__ unsigned long long acctL;          // reference source bytes counted by this workgroup\n",
     "    __shared__ unsigned long long acctL;          // reference source bytes counted by this workgroup\n    __shared__ unsigned long long phL[64];\n"),
    ("backend_hip.hip", "        if (tid == 0)\n            acctL = 0;\n",
     "        if (tid == 0)\n            acctL = 0;\n        if (tid < 64)\n            phL[tid] = 0;\n"),
    ("backend_hip.hip", "    PHASE_MARK(6, kclk);\n",
     "    PHASE_MARK(6, kclk);\n    if (tid < 64 && phL[tid])\n        atomicAdd(&g_phaseClk[tid], phL[tid]);\n"),
]
