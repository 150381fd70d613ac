"""tools/vendor_gemm.py -- the vendor library's GEMM at k_cost_topk's shape, as a
known-good ceiling reference for the contraction (cdna_hip_programming.md
§5.4 rule 10: a ceiling claim needs a reference measured on the same box).

C3 contraction: C^T[n, p] = sum_m Lt[n, m] * WA[p, m], n < 10,240 (nodes,
padded), m < 10,240 (K), p < 102,400 (pods).  The library computes the plain
product and writes it to HBM (int32: 4.2 GB, bf16: 2.1 GB); k_cost_topk
computes the same product and reduces it to per-pod top-8 lists in registers.
So the library time is a ceiling reference for the MFMA loop only, not a like-
for-like kernel: its output store adds ~0.5 ms (int32) at HBM speed.

  torch._int_mm (i8 x i8 -> i32, hipBLASLt on ROCm) and torch.matmul (bf16 ->
  bf16 out, fp32 accumulate), operands: C3-like value ranges (latency 0..105,
  traffic mostly 0..2) and full-range random, HIP events, median of reps.

  python tools/vendor_gemm.py [--pods 102400] [--reps 10]

Prints one JSON line.  Not product code: a measurement aid.
"""
import argparse
import json

import torch

PEAK_I8 = 5033.2e12
PEAK_BF16 = 2516.6e12


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2], ts[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=10240)
    ap.add_argument("--k", type=int, default=10240)
    ap.add_argument("--pods", type=int, default=102400)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    M, K, P = args.nodes, args.k, args.pods
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(0x4E4153)
    out = {"shape": {"M_nodes": M, "K": K, "N_pods": P}, "ops": 2.0 * M * K * P}
    ops = 2.0 * M * K * P

    def fill_i8(rows, cols, lo, hi):
        return torch.randint(lo, hi + 1, (rows, cols), generator=g, device=dev,
                             dtype=torch.int32).to(torch.int8)

    for name, (alo, ahi, blo, bhi) in (("c3_like", (0, 105, 0, 2)),
                                       ("random", (-128, 127, -128, 127))):
        A = fill_i8(M, K, alo, ahi)              # Lt [nodes][K], row-major
        Bt = fill_i8(P, K, blo, bhi)             # WA [pods][K], row-major
        B = Bt.t()                               # [K][pods], column-major view
        rec = {}
        for layout, bb in (("B_colmajor", B), ("B_rowmajor", None)):
            try:
                if bb is None:
                    bb = B.contiguous()
                med, mn = timed(lambda: torch._int_mm(A, bb), args.reps)
                rec[f"int8_{layout}"] = {"ms": med, "ms_min": mn, "tops": ops / med / 1e9,
                                         "frac_int8_peak": ops / (med * 1e-3) / PEAK_I8}
            except Exception as e:  # noqa: BLE001 -- report what the library refuses
                rec[f"int8_{layout}"] = {"error": str(e)[:200]}
            finally:
                torch.cuda.empty_cache()
        Ab, Bb = A.to(torch.bfloat16), Bt.to(torch.bfloat16).t()
        del A, Bt, B
        torch.cuda.empty_cache()
        try:
            med, mn = timed(lambda: torch.matmul(Ab, Bb), args.reps)
            rec["bf16"] = {"ms": med, "ms_min": mn, "tflops": ops / med / 1e9,
                           "frac_bf16_peak": ops / (med * 1e-3) / PEAK_BF16}
        except Exception as e:  # noqa: BLE001
            rec["bf16"] = {"error": str(e)[:200]}
        del Ab, Bb
        torch.cuda.empty_cache()
        out[name] = rec
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
