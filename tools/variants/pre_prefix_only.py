# timing variant: k_solve_pre runs only the prefix passes (wrong outputs)
PATCHES = [("backend_hip.hip", "hipLaunchKernelGGL(k_solve_pre, dim3(2 * solveCount), dim3(kPreThreads), (size_t)solve_pre_lds_bytes(rowsCap),\n                           g_stream, solves + solveBegin, rows, coef, results, acctL, solveCount, 0u);",
            "hipLaunchKernelGGL(k_solve_pre, dim3(solveCount), dim3(kPreThreads), (size_t)solve_pre_lds_bytes(rowsCap),\n                           g_stream, solves + solveBegin, rows, coef, results, acctL, solveCount, 2u);")]
