"""Round 6: per-call host times of the headline call (A^6 * A on 30^3) after W warm-up calls, and the
closing stream sync, to find the fixed cost a 20-step timed region pays that a 200-step one amortises."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench
import slat
ctx = slat.Context(0)
A, P = bench.build_inputs(30, 7, ctx)
for W in (5, 5, 50, 200):
    for _ in range(W):
        P.matmul(A).nnz()
    ctx.sync()
    ts, dev = [], []
    t0 = time.perf_counter()
    for _ in range(20):
        t = time.perf_counter()
        C = P._spgemm(A, slat.FLAG_TIMING) if os.environ.get("PROBE_TIMING") else P.matmul(A)
        C.nnz(); del C
        ts.append((time.perf_counter() - t) * 1e6)
        if os.environ.get("PROBE_TIMING"):
            dev.append(ctx.stats()["total_ms"] * 1e3)
    t = time.perf_counter()
    ctx.sync()
    ts_sync = (time.perf_counter() - t) * 1e6
    tot = (time.perf_counter() - t0) * 1e6
    print(f"W={W} total {tot:.0f} us, per call {tot/20:.1f}; calls " + " ".join(f"{x:.0f}" for x in ts) + f"; sync {ts_sync:.0f}")
    if dev:
        print("   device us " + " ".join(f"{x:.0f}" for x in dev) + f"; mean {sum(dev)/len(dev):.1f}")
