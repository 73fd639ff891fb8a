// ed_split.hpp — two-segment stored H·v for HBM-sized sectors (round 5).
//
// spMatVec_cc (ED_HAMILTONIAN_STORED_HxV.f90:132-143) sums each row of the
// stored H in insertion order.  A one-pass kernel must gather v[col] for every
// element of a row where it processes the row; the down-spin (cross-block)
// elements of an Nlevels=28 sector reach V rows all over the 94 MB vector, and
// no row order keeps their neighbourhood inside an XCD's 4 MB L2 (DESIGN.md
// §2: one-pass traffic >= 1.17x the kernel's own bytes for ANY row order).
// Two passes over a re-laid stored matrix fetch every V line once per pass:
//
//   segment A (k_spmv_pk on the A words, row order): the diagonal and the
//     in-block elements (target state with the row's down pattern idw: the
//     same DimUp-long V row) -> y;
//   segment B (k_spmv_sb, column-chunk order): the cross-block elements of
//     <= 64 consecutive rows of one block (a B slice), added to y -> Hv, with
//     the Lanczos epilogues fused.  B slices are walked chunk-major: XCD x
//     takes the chunks c = x, x+8, ... of every block, so the rows one XCD
//     works on at a time read V[:, 64c : 64c+64] (DimDw x 512 B at N28:
//     1.8 MB), which stays in its L2.
//
// The B elements of a slice that every lane has with the same column offset
// and value (the down-spin hops of normal and nonSU2 sectors: target
// (idw', same up rank), same Jordan-Wigner sign, same value) are stored once
// per slice as a U entry {col - row, dictionary index}: a wave-uniform scalar
// load and one coalesced 512-B gather.  The rest (spin flips, Jx/Jp, pair
// terms) stay per lane as packed words {col:24 | index:8} (L words).  The
// re-lay is lossless: every stored element appears exactly once, with the
// stored double, and the build checks the element count.
//
// Summation order: diagonal, in-block elements in insertion order, then U,
// then L elements — a reordering of spMatVec_cc's row sum (parity 1e-13
// relative, tests/test_gpu_split.py; ED_OPT_STORED_EXACT keeps the one-pass
// bit-identical kernel).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ed_kernels.hpp"

namespace edg {

// One B slice: n <= 64 consecutive rows [row0, row0 + n) of one idw block.
struct SplitSlice {
  int32_t row0;
  int32_t n;
  int32_t nu;    // U entries
  int32_t wl;    // L words per lane (slots)
  int64_t uoff;  // first U entry
  int64_t loff;  // first L word (the slice's 64 * wl words, slot-major)
};
constexpr int kSplitFarMax = 32;   // cross-block elements per row the build handles
constexpr int kSplitGrid = 2048;   // k_spmv_sb blocks (a multiple of 8: one list per XCD)

// ---- build: segment A
// nA[i] = in-block elements of row i; widthA[s] = max over slice s.  Also the
// largest cross-block count of any row (atomicMax into *farmax).
static __global__ void __launch_bounds__(kBlock) k_split_count_a(const int64_t* __restrict__ sptr,
                                                          const uint32_t* __restrict__ words,
                                                          const uint16_t* __restrict__ cnt,
                                                          const uint32_t* __restrict__ map, int ns,
                                                          int64_t dim, int64_t nslice, uint16_t* __restrict__ na,
                                                          int32_t* __restrict__ widthA, int* farmax) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nslice * 64;
       i += (int64_t)gridDim.x * kBlock) {
    int c = 0, f = 0;
    if (i < dim) {
      const uint32_t blk = map[i] >> ns;
      const uint32_t* wp = words + sptr[i >> 6] + (i & 63);
      const int n = cnt[i];
      for (int k = 0; k < n; k++) {
        const uint32_t col = wp[64 * k] & kPackColMask;
        if ((map[col] >> ns) == blk) c++;
        else f++;
      }
      na[i] = (uint16_t)c;
    }
    const int w = wave_max(c);
    const int fm = wave_max(f);
    if ((threadIdx.x & 63) == 0) {
      widthA[i >> 6] = w;
      atomicMax(farmax, fm);
    }
  }
}

static __global__ void __launch_bounds__(kBlock) k_split_fill_a(const int64_t* __restrict__ sptr,
                                                         const uint32_t* __restrict__ words,
                                                         const uint16_t* __restrict__ cnt,
                                                         const uint32_t* __restrict__ map, int ns,
                                                         int64_t dim, int64_t nslice,
                                                         const int64_t* __restrict__ sptrA,
                                                         uint32_t* __restrict__ wordsA, uint32_t zpad) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nslice * 64;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t s = i >> 6;
    const int wA = (int)((sptrA[s + 1] - sptrA[s]) >> 6);
    uint32_t* ap = wordsA + sptrA[s] + (i & 63);
    int k2 = 0;
    if (i < dim) {
      const uint32_t blk = map[i] >> ns;
      const uint32_t* wp = words + sptr[s] + (i & 63);
      const int n = cnt[i];
      for (int k = 0; k < n; k++) {
        const uint32_t wd = wp[64 * k];
        if ((map[wd & kPackColMask] >> ns) == blk) ap[64 * (k2++)] = wd;
      }
    }
    // padding: own column (or 0 past the last row), the dictionary's zero
    const uint32_t pad = (uint32_t)(i < dim ? i : 0) | zpad;
    for (; k2 < wA; k2++) ap[64 * k2] = pad;
  }
}

// ---- build: segment B (one wavefront per slice).  FILL = false: nu, wl per
// slice; FILL = true: the U list and the L words at the slice's offsets.
// The lane's cross-block elements are staged in LDS as 64-bit keys
// {col - row : 32 | dictionary index : 32}; an element of lane 0 is uniform
// when every active lane holds the same key.
template <bool FILL>
__global__ void __launch_bounds__(kBlock) k_split_b(const int64_t* __restrict__ sptr,
                                                   const uint32_t* __restrict__ words,
                                                   const uint16_t* __restrict__ cnt,
                                                   const uint32_t* __restrict__ map, int ns,
                                                   SplitSlice* __restrict__ sl, int64_t nsl,
                                                   int2* __restrict__ ul, uint32_t* __restrict__ lw,
                                                   uint32_t zpad) {
  __shared__ unsigned long long keys[kBlock / 64][kSplitFarMax][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t q = (int64_t)blockIdx.x * (kBlock / 64) + wv; q < nsl; q += (int64_t)gridDim.x * (kBlock / 64)) {
    const int qq = __builtin_amdgcn_readfirstlane((int)q);
    const SplitSlice S = sl[qq];
    const bool on = lane < S.n;
    const int64_t i = S.row0 + (on ? lane : 0);
    int nf = 0;
    if (on) {
      const uint32_t blk = map[i] >> ns;
      const uint32_t* wp = words + sptr[i >> 6] + (i & 63);
      const int n = cnt[i];
      for (int k = 0; k < n && nf < kSplitFarMax; k++) {
        const uint32_t wd = wp[64 * k];
        const uint32_t col = wd & kPackColMask;
        if ((map[col] >> ns) != blk)
          keys[wv][nf++][lane] = ((unsigned long long)(uint32_t)((int32_t)col - (int32_t)i) << 32) |
                                 (wd >> kPackShift);
      }
    }
    const int nf0 = __builtin_amdgcn_readfirstlane(nf);  // lane 0 is always active
    uint32_t used = 0;
    int nu = 0;
    for (int k0 = 0; k0 < nf0; k0++) {
      const unsigned long long key = keys[wv][k0][0];
      int pos = -1;
      for (int j = 0; j < nf; j++)
        if (keys[wv][j][lane] == key) pos = j;
      const bool all = __ballot(!on || pos >= 0) == __ballot(1);
      if (all) {
        if (on) used |= 1u << pos;
        if constexpr (FILL) {
          if (lane == 0) ul[S.uoff + nu] = make_int2((int32_t)(key >> 32), (int32_t)(key & 0xffu));
        }
        nu++;
      }
    }
    const int nl = nf - __popc(used);
    if constexpr (!FILL) {
      const int wl = wave_max(on ? nl : 0);
      if (lane == 0) {
        sl[qq].nu = nu;
        sl[qq].wl = wl;
      }
    } else {
      uint32_t* lp = lw + S.loff + lane;
      int k2 = 0;
      for (int j = 0; j < nf; j++)
        if (!((used >> j) & 1u)) {
          const unsigned long long kk = keys[wv][j][lane];
          lp[64 * (k2++)] = (uint32_t)((int32_t)i + (int32_t)(kk >> 32)) | ((uint32_t)(kk & 0xffu) << kPackShift);
        }
      for (; k2 < S.wl; k2++) lp[64 * k2] = (uint32_t)i | zpad;
    }
  }
}

// ---- segment B H·v: y (segment A's rows) + the slice's cross-block
// elements -> epilogue.  One wavefront per slice; XCD x walks its own list
// [xoff[x], xoff[x+1]) (chunk-major) with the blocks dealt to it.
constexpr int kSplitChunk = 8;
template <bool HC, bool VC, int NT, class Epi>
__global__ void __launch_bounds__(kBlock) k_spmv_sb(const SplitSlice* __restrict__ sl, const int* __restrict__ xoff,
                                                    const int2* __restrict__ ul, const uint32_t* __restrict__ lw,
                                                    const val_t<HC>* __restrict__ dict,
                                                    const val_t<VC>* __restrict__ x, const val_t<VC>* y, Epi epi) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  if (epi.skip()) return;
  epi.prepare();
  __shared__ H sdict[256];
  sdict[threadIdx.x] = dict[threadIdx.x];  // kBlock == 256 == dictionary capacity
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int xcd = blockIdx.x & 7, g8 = gridDim.x >> 3;
  const int lo = xoff[xcd], hi = xoff[xcd + 1];
  double part = 0.0;
  for (int q = lo + (int)(blockIdx.x >> 3) * (kBlock / 64) + wv; q < hi; q += g8 * (kBlock / 64)) {
    const SplitSlice S = sl[q];
    const bool on = lane < S.n;
    const int i = S.row0 + (on ? lane : 0);
    V acc = y[i];
    const int2* up = ul + S.uoff;
    for (int k0 = 0; k0 < S.nu; k0 += kSplitChunk) {
      int2 e[kSplitChunk];
      V g[kSplitChunk];
#pragma unroll
      for (int k = 0; k < kSplitChunk; k++) e[k] = k0 + k < S.nu ? up[k0 + k] : make_int2(0, 0);
#pragma unroll
      for (int k = 0; k < kSplitChunk; k++) g[k] = x[i + e[k].x];
#pragma unroll
      for (int k = 0; k < kSplitChunk; k++)
        if (k0 + k < S.nu) acc = add(acc, mul(sdict[e[k].y], g[k]));
    }
    const uint32_t* wp = lw + S.loff + lane;
    for (int k0 = 0; k0 < S.wl; k0 += kSplitChunk) {
      uint32_t c[kSplitChunk];
      V g[kSplitChunk];
#pragma unroll
      for (int k = 0; k < kSplitChunk; k++) c[k] = k0 + k < S.wl ? ldm<NT>(wp + 64 * (k0 + k)) : (uint32_t)i;
#pragma unroll
      for (int k = 0; k < kSplitChunk; k++) g[k] = x[c[k] & kPackColMask];
#pragma unroll
      for (int k = 0; k < kSplitChunk; k++)
        if (k0 + k < S.wl) acc = add(acc, mul(sdict[c[k] >> kPackShift], g[k]));
    }
    if (on) part += epi.row((int64_t)i, acc, x[i]);
  }
  epi.finish(part);
}

}  // namespace edg
