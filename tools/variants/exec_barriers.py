# profiling variant: every barrier of k_exec timed per wave.  For barrier n
# (in source order), g_phaseClk[n] sums the waves' work since their previous
# barrier and g_phaseClk[32 + n] their wait at barrier n (lane 0 of each
# wave, LDS accumulators flushed once per workgroup).  The barrier lines are
# printed by the build.  Build with
#   python tools/variant_src.py barriers tools/variants/exec_barriers.py -DSGPU_PHASE_CLOCKS
import re

BARRIER_LINES = []


def transform(name, text):
    if name != "backend_hip.hip":
        return text
    a = text.index("__global__ __launch_bounds__(kExecThreads) void k_exec(")
    b = text.index("// Triangular solve", a)
    body = text[a:b]
    n = [0]

    def sub(m):
        k = n[0]
        n[0] += 1
        return "SGPU_BAR(%d);" % k

    body = re.sub(r"__syncthreads\(\);", sub, body)
    assert n[0] <= 32, n[0]
    # accumulators and the per-wave clock
    body = body.replace(
        "    __shared__ unsigned long long acctL;          // reference source bytes counted by this workgroup\n",
        "    __shared__ unsigned long long acctL;          // reference source bytes counted by this workgroup\n"
        "    __shared__ unsigned long long barL[64];\n    unsigned long long barPrev = clock64();\n", 1)
    body = body.replace("        if (tid == 0)\n            acctL = 0;\n",
                        "        if (tid == 0)\n            acctL = 0;\n        if (tid < 64)\n            barL[tid] = 0;\n", 1)
    body = body.replace("    PHASE_MARK(6, kclk);\n",
                        "    PHASE_MARK(6, kclk);\n    __syncthreads();\n    if (tid < 63 && barL[tid])\n"
                        "        atomicAdd(&g_phaseClk[tid], barL[tid]);\n    if (tid == 0)\n"
                        "        atomicAdd(&g_phaseClk[63], 1ull);\n", 1)
    macro = """
#define SGPU_BAR(k)                                                                        \\
    do {                                                                                   \\
        const unsigned long long ta_ = clock64();                                          \\
        __syncthreads();                                                                   \\
        const unsigned long long tb_ = clock64();                                          \\
        if ((threadIdx.x & 63) == 0) {                                                     \\
            atomicAdd(&barL[k], ta_ - barPrev);                                            \\
            atomicAdd(&barL[32 + (k)], tb_ - ta_);                                         \\
        }                                                                                  \\
        barPrev = clock64();                                                               \\
    } while (0)
"""
    # per-unit clocks of the update phase and the row tasks (lane 0 of each
    # wave): barL[11..13] version / update / plan units, [14..16] their
    # counts, [17]/[18] planned-row quad tasks, [19]/[20] general rows
    L0 = "if ((threadIdx.x & 63) == 0) "
    for old, new in [
        ("PHASE_ADD(26, PHASE_CLK() - vclk0);", L0 + "atomicAdd(&barL[11], clock64() - vclk0);"),
        ("PHASE_ADD(19, PHASE_CLK() - uclk0);", L0 + "atomicAdd(&barL[12], clock64() - uclk0);"),
        ("PHASE_ADD(20, PHASE_CLK() - pclk0);", L0 + "atomicAdd(&barL[13], clock64() - pclk0);"),
        ("PHASE_ADD(29, 1);", L0 + "atomicAdd(&barL[14], 1ull);"),
        ("PHASE_ADD(27, 1);", L0 + "atomicAdd(&barL[15], 1ull);"),
        ("PHASE_ADD(28, 1);", L0 + "atomicAdd(&barL[16], 1ull);"),
        ("PHASE_MARK(15, qclk);", L0 + "{ atomicAdd(&barL[17], clock64() - qclk); atomicAdd(&barL[18], 1ull); }"),
        ("PHASE_MARK(22, rclk);", L0 + "{ atomicAdd(&barL[19], clock64() - rclk); atomicAdd(&barL[20], 1ull); }"),
    ]:
        assert old in body, old
        body = body.replace(old, new, 1)
    # (PHASE_MARK / PHASE_ADD and the op counters off: only the barrier clocks)
    body = body.replace("g_phaseClk", "g_dummyClk").replace("&g_dummyClk[tid], barL[tid]", "&g_phaseClk[tid], barL[tid]")
    off = ("#undef PHASE_MARK\n#define PHASE_MARK(k, t) (void)0\n#undef PHASE_ADD\n#define PHASE_ADD(k, v) (void)0\n"
           "__device__ unsigned long long g_dummyClk[64];\n")
    r = text.index("__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane)")
    text = text[:r] + off + text[r:a] + macro + body + text[b:]
    out = text
    # record barrier line numbers for the report
    for i, ln in enumerate(out.split("\n")):
        mm = re.search(r"SGPU_BAR\((\d+)\);", ln)
        if mm and "define" not in ln:
            BARRIER_LINES.append((int(mm.group(1)), i + 1))
    open("vbuild_barrier_lines.txt", "w").write("\n".join("%d %d" % x for x in BARRIER_LINES))
    return out
