"""Measurement-only kernel variants for A/B runs on the GPU box.

Builds a variant of libsvdj_hip.so from a PATCHED COPY of csrc/hip/block.hip
(the production source never carries experiment switches).  Variants:

  nogram    the cross-Gram launches of the cross steps are dropped: the EVD
            reads the previous step's slabs (valid Grams of other pairs, so the
            rotations stay orthogonal and nothing is skipped).  A sweep then
            costs what it would if the Gram were free.
  fused     nogram + the Gram's matrix-core work added to the A part of the
            apply: 64 extra MFMAs per 32-row tile and pair (the W x W cross
            product of the tile's rows: +25 % on A rows, +12.5 % overall), 64
            more accumulator registers.  An optimistic model of a fused
            apply+Gram kernel (VERDICT r2 "remove an HBM pass on 1 GPU"): it
            leaves out the re-ordering of the row work that fusion needs
            (next-step pairs span two current pairs) and the slab writes.
  fusedl2   nogram + the work a fused fp32 W=64 apply would add: after its
            stores, each wave re-reads its tile's X and Y rows in Gram operand
            layout (the apply's accumulators hold rows on lanes, the Gram needs
            columns on lanes) and runs the 64 MFMAs of their W x W product.
            Models the operand traffic and register pressure of fusion, not
            the cross-pair re-ordering.
  apply384  fp32 W=64 apply with 6 waves per workgroup and at most 168
            registers (3 waves per SIMD instead of 2; one Q fill per 6 waves).
  gram3     fp32 W=64 cross Gram with 8 rows per lane and at most 168
            registers (3 waves per SIMD instead of 2).

The nogram/fused results are wrong by construction; only the timing of
`bench.py --simulate-P P --sim-sweeps 2` (full-work sweeps) is meaningful.
Usage: python tools/kernel_ab.py VARIANT OUT.so
"""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "svd-jacobi-mpi-cuda_amd"
CSRC = PKG / "csrc"

GRAM_CROSS = """  } else {
    hipLaunchKernelGGL((gram_kernel<T, W, GRAM_CROSS>)"""

APPLY_TAIL = """        dst[(size_t)M::acc_row_uni(e) * ld + (st_off + (uint32_t)r0)] = acc[e];
    }
    if (!more) break;"""

FUSED_TAIL = """        dst[(size_t)M::acc_row_uni(e) * ld + (st_off + (uint32_t)r0)] = acc[e];
    }
    if (base == A) {  // fusion-bound model: the W x W cross product of this tile
      typename M::acc_t g[4] = {M::zero(), M::zero(), M::zero(), M::zero()};
#pragma unroll
      for (int i = 0; i < NK / 4; ++i)
#pragma unroll
        for (int t = 0; t < 4; ++t) g[t] = M::mfma(xv[4 * i + t], xv[NK - 1 - 4 * i - t], g[t]);
      if (lda == 0x7fffffff)  // never true: keeps the products alive
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int e = 0; e < M::NACC; ++e) A[t * M::NACC + e] = g[t][e];
    }
    if (!more) break;"""

FUSEDL2_TAIL = """        dst[(size_t)M::acc_row_uni(e) * ld + (st_off + (uint32_t)r0)] = acc[e];
    }
    if constexpr (sizeof(T) == 4 && W == 64) {
      if (base == A) {  // fusion model: the tile's W x W cross product, re-read
        __builtin_amdgcn_s_waitcnt(0);
        typename M::acc_t g[4] = {M::zero(), M::zero(), M::zero(), M::zero()};
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          T xa[2][8], yb[2][8];
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const size_t off = (size_t)(c * 32 + lc) * ld + r0 + kg * 16 + hf * 8;
            load_col16B<T, 8>(xi + off, xa[c]);
            load_col16B<T, 8>(xj + off, yb[c]);
          }
#pragma unroll
          for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
              for (int b = 0; b < 2; ++b) g[2 * a + b] = M::mfma(xa[a][t], yb[b][t], g[2 * a + b]);
        }
        if (lda == 0x7fffffff)  // never true: keeps the products alive
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int e = 0; e < M::NACC; ++e) A[t * M::NACC + e] = g[t][e];
      }
    }
    if (!more) break;"""

APPLY_THREADS = "constexpr int apply_threads() { return kApplyThreads; }"
APPLY_DECL = "__global__ __launch_bounds__((apply_threads<T, W>())) void apply_kernel("
GRAM_LPL = "constexpr int kGramLpl64 = 16;"
GRAM_DECL = "__global__ __launch_bounds__(kGramThreads) void gram_kernel("


def _sub(src: str, old: str, new: str) -> str:
    assert src.count(old) == 1, f"patch anchor not found once: {old[:60]!r}"
    return src.replace(old, new)


def patch(src: str, variant: str) -> str:
    if variant in ("nogram", "fused", "fusedl2"):
        src = _sub(src, GRAM_CROSS, GRAM_CROSS.replace("} else {", "} else if (false) {"))
    if variant == "fused":
        src = _sub(src, APPLY_TAIL, FUSED_TAIL)
    if variant == "fusedl2":
        src = _sub(src, APPLY_TAIL, FUSEDL2_TAIL)
    if variant == "apply384":
        src = _sub(src, APPLY_THREADS, "constexpr int apply_threads() { return (sizeof(T) == 4 && W == 64) ? 384 : kApplyThreads; }\n"
                   "template <typename T, int W>\n"
                   "__host__ __device__ constexpr int apply_wpe() { return (sizeof(T) == 4 && W == 64) ? 3 : 1; }")
        src = _sub(src, APPLY_DECL, "__global__ __launch_bounds__((apply_threads<T, W>())) "
                   "__attribute__((amdgpu_waves_per_eu(apply_wpe<T, W>()))) void apply_kernel(")
    if variant == "gram3":
        src = _sub(src, GRAM_LPL, "constexpr int kGramLpl64 = 8;\n"
                   "template <typename T, int W, int MODE>\n"
                   "__host__ __device__ constexpr int gram_wpe() { return (sizeof(T) == 4 && W == 64 && MODE == 0) ? 3 : 1; }")
        src = _sub(src, GRAM_DECL, "__global__ __launch_bounds__(kGramThreads) "
                   "__attribute__((amdgpu_waves_per_eu(gram_wpe<T, W, MODE>()))) void gram_kernel(")
    return src


VARIANTS = ("nogram", "fused", "fusedl2", "apply384", "gram3")


def main():
    variant, out = sys.argv[1], Path(sys.argv[2]).resolve()
    if variant not in VARIANTS:
        raise SystemExit("variant: " + " | ".join(VARIANTS))
    scratch = out.parent / f"ab_{variant}"
    scratch.mkdir(parents=True, exist_ok=True)
    blk = scratch / "block.hip"
    blk.write_text(patch((CSRC / "hip" / "block.hip").read_text(), variant))
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-unused-result",
             "-Wno-pass-failed", f"-I{CSRC / 'include'}", f"-I{CSRC / 'hip'}"]
    objs = []
    for src in (blk, CSRC / "hip" / "post.hip", CSRC / "hip" / "scalar.hip"):
        obj = scratch / (src.stem + ".o")
        subprocess.run(["hipcc", *flags, "-c", str(src), "-o", str(obj)], check=True)
        objs.append(str(obj))
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", str(out)],
                   check=True)
    print(f"built {variant} -> {out}")


if __name__ == "__main__":
    main()
