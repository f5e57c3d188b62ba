"""Phase breakdown of the bench workload, device-resident vs end-to-end
(pinned host originals in, every output gathered back):
    python tools/e2e_probe.py [steps]
Prints ms per step and the harness phases (create/step/flush/resolve/finish)
for both modes, so the cost of the transfers shows up by phase."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import scenario_lib as S  # noqa: E402
import bench  # noqa: E402


def pcie_rates(nbytes):
    """H2D / D2H GB/s of one pinned copy of `nbytes` (torch, the current GPU)."""
    import time
    import torch
    if not torch.cuda.is_available():
        return None
    h = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    out = []
    for src, dst in ((h, d), (d, h)):
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        out.append(round(3 * nbytes / (time.perf_counter() - t) / 1e9, 1))
    return out


def main():
    print("pinned H2D/D2H GB/s (367 MB):", pcie_rates(367 << 20), flush=True)
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    lib = os.environ.get("SGPU_LIB", os.path.join(ROOT, "siamese_amd", "libsiamese_amd.so"))
    cfg = bench.workload(0, 1024)
    sess = S.BatchSession(lib, cfg, device=0 if "null" not in lib else -1)
    try:
        for e2e in (False, True):
            sess.run(steps=2, warmup=0, verify=False, threads=0, groups=4, e2e=e2e, digest=False)
            res, rep = sess.run(steps=steps, warmup=0, verify=False, threads=0, groups=4, e2e=e2e,
                                digest=False)
            if any(r.status for r in res):
                raise SystemExit("probe run failed (e2e=%s)" % e2e)
            ph = [round(x / steps * 1e3, 3) for x in rep.phase_seconds]
            print("e2e=%d ms/step %.3f device %.3f phases create/step/flush/resolve/finish %s" % (
                e2e, rep.seconds / steps * 1e3, rep.device_ms / steps, ph), flush=True)
    finally:
        sess.close()


if __name__ == "__main__":
    main()
