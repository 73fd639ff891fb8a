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
//     <= 128 consecutive rows of one block (a B slice), added to y -> Hv,
//     with the Lanczos epilogues fused.  B slices are walked chunk-major
//     (chunk c = in-block rows [128c, 128c + 128) of every block) and the
//     list is cut into eight contiguous parts, one per XCD, so the rows one
//     XCD works on at a time read V[:, 128c : 128c+128] (DimDw x 1 KB at
//     N28: 3.5 MB), which stays in its L2.
//
// The B elements of a slice that every lane has with the same column offset
// and value (the down-spin hops of normal and nonSU2 sectors: target
// (idw', same up rank), same Jordan-Wigner sign, same value) are stored once
// per slice as a U entry {col - row, dictionary index}: a wave-uniform scalar
// load and one coalesced 1-KB gather (16 B per lane).  The rest (spin flips, Jx/Jp, pair
// terms) stay per lane as packed words {col:24 | index:8} (L words).  The
// re-lay is lossless: every stored element appears exactly once, with the
// stored double (sector info reports the cross-block count and its U share).
//
// Summation order: diagonal, in-block elements in insertion order, then U,
// then L elements — a reordering of spMatVec_cc's row sum (parity 1e-13
// relative, tests/test_gpu_split.py; ED_OPT_STORED_EXACT keeps the one-pass
// bit-identical kernel).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ed_kernels.hpp"

#ifndef ED_SA_R
#define ED_SA_R 2
#endif

namespace edg {

// One B slice: n <= kSplitRows consecutive rows [row0, row0 + n) of one idw
// block.  L words slot-major: word k of row row0 + r at loff + 128 k + r.
// (all fields 32- or 64-bit: the kernel reads a slice with scalar loads)
struct SplitSlice {
  int32_t row0;
  int32_t nfl;   // rows n | flags << 16 (kSplitPair: row0, n and every U column offset even)
  int32_t nu;    // U entries, padded to a multiple of kSplitChunk with {0, zero value}
  int32_t wl;    // L words per row (slots), padded to a multiple of kSplitLChunk
  int64_t uoff;  // first U entry
  int64_t loff;  // first L word (the slice's kSplitRows * wl words, slot-major)
};
constexpr int kSplitFarMax = 32;   // cross-block elements per row the build handles
constexpr int kSplitRows = 128;    // rows per B slice (two per lane)
constexpr int kSplitPair = 1;      // SplitSlice flag: 16-byte pair gathers apply
constexpr int kSplitChunk = 8;     // U elements per load batch (U lists padded to it)
constexpr int kSplitLChunk = 4;    // L slots per load batch (L widths padded to it)
__host__ __device__ inline int split_n(const SplitSlice& q) { return q.nfl & 0xffff; }
__host__ __device__ inline int split_flags(const SplitSlice& q) { return q.nfl >> 16; }
constexpr int kSplitAGrid = 2048;  // k_spmv_sa blocks (a multiple of 8: one slice range per XCD)
constexpr int kSplitGrid = 1280;   // k_spmv_sb blocks (a multiple of 8: one list per XCD; pass D's grid)

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

// ---- build: segment B (one wavefront per slice of <= 128 rows, two
// adjacent rows per lane).  FILL = false: nu, wl per slice; FILL = true: the
// U list and the L words at the slice's offsets.  Each row's cross-block
// elements are staged in LDS as 64-bit keys {col - row : 32 | dictionary
// index : 32}; an element of the slice's first row is uniform when every
// row of the slice holds the same key.
constexpr int kSplitBuildBlock = 128;  // 2 waves: 2 x 32 x 128 keys = 64 KB of LDS
template <bool FILL>
__global__ void __launch_bounds__(kSplitBuildBlock) k_split_b(const int64_t* __restrict__ sptr,
                                                             const uint32_t* __restrict__ words,
                                                             const uint16_t* __restrict__ cnt,
                                                             const uint32_t* __restrict__ map, int ns,
                                                             SplitSlice* __restrict__ sl, int64_t nsl,
                                                             int2* __restrict__ ul, uint32_t* __restrict__ lw,
                                                             uint32_t zpad) {
  constexpr int NW = kSplitBuildBlock / 64;
  __shared__ unsigned long long keys[NW][kSplitFarMax][kSplitRows];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t q = (int64_t)blockIdx.x * NW + wv; q < nsl; q += (int64_t)gridDim.x * NW) {
    const int qq = __builtin_amdgcn_readfirstlane((int)q);
    const SplitSlice S = sl[qq];
    int nf[2] = {0, 0};
    bool on[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int r = 2 * lane + h;
      on[h] = r < split_n(S);
      if (!on[h]) continue;
      const int64_t i = S.row0 + r;
      const uint32_t blk = map[i] >> ns;
      const uint32_t* wp = words + sptr[i >> 6] + (i & 63);
      const int n = cnt[i];
      for (int k = 0; k < n && nf[h] < kSplitFarMax; k++) {
        const uint32_t wd = wp[64 * k];
        const uint32_t col = wd & kPackColMask;
        if ((map[col] >> ns) != blk)
          keys[wv][nf[h]++][r] = ((unsigned long long)(uint32_t)((int32_t)col - (int32_t)i) << 32) |
                                 (wd >> kPackShift);
      }
    }
    const int nf0 = __builtin_amdgcn_readfirstlane(nf[0]);  // row 0 of the slice always exists
    uint32_t used[2] = {0u, 0u};
    int nu = 0;
    bool even = true;  // every U column offset even
    for (int k0 = 0; k0 < nf0; k0++) {
      const unsigned long long key = keys[wv][k0][0];
      // the first not yet matched slot with this key: a row holding the same
      // (col, value) key twice matches it once per occurrence (k_fill does
      // not merge duplicate columns the way sp_insert_element would)
      int pos[2] = {-1, -1};
#pragma unroll
      for (int h = 0; h < 2; h++)
        for (int j = nf[h] - 1; j >= 0; j--)
          if (!((used[h] >> j) & 1u) && keys[wv][j][2 * lane + h] == key) pos[h] = j;
      const bool mine = (!on[0] || pos[0] >= 0) && (!on[1] || pos[1] >= 0);
      if (__ballot(mine) == __ballot(1)) {
#pragma unroll
        for (int h = 0; h < 2; h++)
          if (on[h]) used[h] |= 1u << pos[h];
        if constexpr (FILL) {
          if (lane == 0) ul[S.uoff + nu] = make_int2((int32_t)(key >> 32), (int32_t)(key & 0xffu));
        }
        even = even && !((key >> 32) & 1u);
        nu++;
      }
    }
    const int nl = max(on[0] ? nf[0] - __popc(used[0]) : 0, on[1] ? nf[1] - __popc(used[1]) : 0);
    if constexpr (FILL) {
      // pad the U list to the slice's (padded) count with {0, zero value}
      for (int k = nu + lane; k < S.nu; k += 64) ul[S.uoff + k] = make_int2(0, (int32_t)(zpad >> kPackShift));
    }
    if constexpr (!FILL) {
      const int wl = wave_max(nl);
      if (lane == 0) {
        const int n = split_n(S);
        sl[qq].nu = nu;
        sl[qq].wl = wl;
        sl[qq].nfl = n | (((even && !(S.row0 & 1) && !(n & 1)) ? kSplitPair : 0) << 16);
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int r = 2 * lane + h;
        const int64_t i = S.row0 + (on[h] ? r : 0);
        uint32_t* lp = lw + S.loff + r;
        int k2 = 0;
        if (on[h])
          for (int j = 0; j < nf[h]; j++)
            if (!((used[h] >> j) & 1u)) {
              const unsigned long long kk = keys[wv][j][r];
              lp[kSplitRows * (k2++)] =
                  (uint32_t)((int32_t)i + (int32_t)(kk >> 32)) | ((uint32_t)(kk & 0xffu) << kPackShift);
            }
        for (; k2 < S.wl; k2++) lp[kSplitRows * k2] = (uint32_t)i | zpad;
      }
    }
  }
}

// ---- segment B H·v: y (segment A's rows) + the slice's cross-block
// elements -> epilogue.  One wavefront per slice of <= 128 rows, lane l
// taking rows 2l and 2l+1.  Pair slices (kSplitPair: row0, n and every U
// column offset even) on a 16-byte aligned real vector gather each U element
// of the two rows with one 16-byte load (as pass D of the two-pass Kronecker
// H·v), branch-free; other slices take two 8-byte (or 16-byte complex)
// gathers per element.  XCD x walks its own part [xoff[x], xoff[x+1]) of the
// chunk-major list with the blocks dealt to it.
// ---- segment A H·v: y = diag .* x + in-block elements, row order.  The
// in-block gathers stay inside the row's own DimUp-long V row, so the rows
// are walked in order: XCD x takes the x-th eighth of the 64-row slices
// (its L2 holds the V rows its neighbouring slices read); a wavefront takes
// R consecutive slices at a time with every load of the R slices in flight
// before the first is summed (a one-row-per-thread grid exposes the
// sptr -> words -> gathers latency chain once per row).
template <bool HC, bool VC, int NT, int CH, int R>
__global__ void __launch_bounds__(kBlock) k_spmv_sa(const val_t<HC>* __restrict__ diag, const int64_t* __restrict__ sptr,
                                                    const uint32_t* __restrict__ words,
                                                    const val_t<HC>* __restrict__ dict,
                                                    const val_t<VC>* __restrict__ x, val_t<VC>* __restrict__ y,
                                                    int64_t dim, int64_t nslice) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  __shared__ H sdict[256];
  sdict[threadIdx.x] = dict[threadIdx.x];  // kBlock == 256 == dictionary capacity
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int xcd = blockIdx.x & 7;
  const int64_t s_lo = nslice * xcd / 8, s_hi = nslice * (xcd + 1) / 8;
  const int64_t nwx = (int64_t)(gridDim.x >> 3) * (kBlock / 64);  // waves per XCD
  for (int64_t s0 = s_lo + R * ((int64_t)(blockIdx.x >> 3) * (kBlock / 64) + wv); s0 < s_hi; s0 += R * nwx) {
    int64_t b[R + 1];
    int w[R];
    int64_t i[R];
    bool ok[R];
#pragma unroll
    for (int r = 0; r <= R; r++) b[r] = sptr[min(s0 + r, s_hi)];
    int wmax = 0;
#pragma unroll
    for (int r = 0; r < R; r++) {
      w[r] = (int)((b[r + 1] - b[r]) >> 6);  // 0 for a slice past s_hi
      wmax = max(wmax, w[r]);
      i[r] = (s0 + r) * 64 + lane;
      ok[r] = s0 + r < s_hi && i[r] < dim;
      if (!ok[r]) i[r] = s0 * 64;            // a valid row (row s0*64 < dim)
    }
    V xi[R], acc[R];
    H dg[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      xi[r] = x[i[r]];
      dg[r] = ldh<NT>(diag + i[r]);
    }
    for (int k0 = 0; k0 < wmax || k0 == 0; k0 += CH) {
      uint32_t c[R][CH];
#pragma unroll
      for (int r = 0; r < R; r++) {
        const uint32_t* wp = words + b[r] + lane;
        if (w[r] > 0) {  // (wave-uniform: one branch per slice, none per slot)
#pragma unroll
          for (int k = 0; k < CH; k++) c[r][k] = ldm<NT>(wp + 64 * min(k0 + k, w[r] - 1));
        } else {
#pragma unroll
          for (int k = 0; k < CH; k++) c[r][k] = (uint32_t)i[r];
        }
      }
      V g[R][CH];
      H h[R][CH];
#pragma unroll
      for (int r = 0; r < R; r++)
#pragma unroll
        for (int k = 0; k < CH; k++) {
          g[r][k] = x[c[r][k] & kPackColMask];
          h[r][k] = sdict[c[r][k] >> kPackShift];
        }
      // every gather issued before the first is used (without this fence the
      // scheduler sinks the complex gathers to their uses: one round trip per
      // element, 0.73 ms per N28 launch instead of ~0.2)
      asm volatile("" ::: "memory");
      if (k0 == 0) {
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = mul(dg[r], xi[r]);
      }
#pragma unroll
      for (int r = 0; r < R; r++)
#pragma unroll
        for (int k = 0; k < CH; k++) acc[r] = sel(k0 + k < w[r], add(acc[r], mul(h[r][k], g[r][k])), acc[r]);
    }
#pragma unroll
    for (int r = 0; r < R; r++)
      if (ok[r]) {
        // a plain (write-back) store: segment B reads y back from the
        // Infinity Cache (segment A's only other cached stream is the
        // gathered x, 94 + 94 MB at N28 real; NT stores: segment B 81 us
        // instead of 59, profiles/r5)
        y[i[r]] = acc[r];
      }
  }
}

typedef double sb_d2 __attribute__((ext_vector_type(2)));
typedef unsigned int sb_u2 __attribute__((ext_vector_type(2)));

// one 128-row slice in the generic form: the lane's two rows apart (8-byte
// gathers), for slices without the pair property
template <bool HC, bool VC, int NT, int UCH, class Epi>
__device__ __forceinline__ double sb_generic(const SplitSlice& S, int lane, const int2* __restrict__ ul,
                                             const uint32_t* __restrict__ lw, const val_t<HC>* sdict,
                                             const val_t<VC>* __restrict__ x, const val_t<VC>* y, Epi& epi) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  const int n = split_n(S);
  const bool on0 = 2 * lane < n, on1 = 2 * lane + 1 < n;
  const int i0 = S.row0 + (on0 ? 2 * lane : 0);  // idle lanes: the slice's first row
  const int i1 = on1 ? i0 + 1 : i0;
  const int2* up = ul + S.uoff;
  const uint32_t* wp = lw + S.loff + 2 * lane;
  V a0 = y[i0], a1 = y[i1];
  for (int k0 = 0; k0 < S.nu; k0 += UCH) {
    int2 e[UCH];
    V g0[UCH], g1[UCH];
#pragma unroll
    for (int k = 0; k < UCH; k++) e[k] = up[k0 + k];  // padded list: whole chunks
#pragma unroll
    for (int k = 0; k < UCH; k++) {
      g0[k] = x[i0 + e[k].x];
      g1[k] = x[i1 + e[k].x];
    }
    asm volatile("" ::: "memory");  // all gathers in flight before the first use
#pragma unroll
    for (int k = 0; k < UCH; k++) {
      const H h = sdict[e[k].y];
      a0 = add(a0, mul(h, g0[k]));
      a1 = add(a1, mul(h, g1[k]));
    }
  }
  for (int k0 = 0; k0 < S.wl; k0 += kSplitLChunk) {
    sb_u2 c[kSplitLChunk];
    V g0[kSplitLChunk], g1[kSplitLChunk];
#pragma unroll
    for (int k = 0; k < kSplitLChunk; k++) c[k] = ldm<NT>((const sb_u2*)(wp + kSplitRows * (k0 + k)));
#pragma unroll
    for (int k = 0; k < kSplitLChunk; k++) {
      g0[k] = x[c[k].x & kPackColMask];
      g1[k] = x[c[k].y & kPackColMask];
    }
#pragma unroll
    for (int k = 0; k < kSplitLChunk; k++) {
      a0 = add(a0, mul(sdict[c[k].x >> kPackShift], g0[k]));
      a1 = add(a1, mul(sdict[c[k].y >> kPackShift], g1[k]));
    }
  }
  double part = 0.0;
  if (on0) part += epi.row((int64_t)i0, a0, x[i0]);
  if (on1) part += epi.row((int64_t)i1, a1, x[i1]);
  return part;
}

// ---- segment B H·v: y (segment A's rows) + the slices' cross-block
// elements -> epilogue.  Slices are walked in 64-row halves, chunk-major
// (half-chunk c = in-block rows [64c, 64c + 64) of every block): the V
// columns one XCD reads at a time are DimDw x 512 B (1.8 MB at N28), which
// stay in its L2 beside the y and Hv streams (128-row chunks: V fetched
// ~2.9x).
//   real vectors: a wavefront takes an item of two halves (of two blocks)
//     with equal U / L counts, 32 lanes each, two adjacent rows per lane:
//     every U element of the two rows is one 16-byte gather (pair slices:
//     kSplitPair), both halves' U lists read with scalar loads and selected
//     per lane group; slices without the pair property go through the
//     generic list, one 128-row slice per wavefront;
//   complex vectors: one half per wavefront, one row (16 B) per lane.
// Returns nothing; the epilogue's partials via epi.finish.
// UCH: U entries per load batch (the U lists are padded to a multiple of it:
// the sector's largest U count when that is 7, else kSplitChunk)
template <bool HC, bool VC, int NT, class Epi, int UCH = kSplitChunk>
__global__ void __launch_bounds__(kBlock) k_spmv_sb(const SplitSlice* __restrict__ sl, const int2* __restrict__ items,
                                                    const int* __restrict__ xoffI, const int* __restrict__ glist,
                                                    const int* __restrict__ xoffG, const int2* __restrict__ ul,
                                                    const uint32_t* __restrict__ lw, const val_t<HC>* __restrict__ dict,
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
  const int w0 = (int)(blockIdx.x >> 3) * (kBlock / 64) + wv, nwx = g8 * (kBlock / 64);
  double part = 0.0;
  if constexpr (!VC) {
    // ---- items: two halves per wavefront, 16-byte pair gathers
    const int grp = lane >> 5, l = lane & 31;
    for (int q = xoffI[xcd] + w0; q < xoffI[xcd + 1]; q += nwx) {
      const int2 it = items[q];
      const bool hasB = it.y >= 0;
      const SplitSlice SA = sl[it.x >> 1];
      const SplitSlice SB = sl[(hasB ? it.y : it.x) >> 1];
      const int nu = SA.nu, wl = SA.wl;  // equal in both halves (build)
      const int half = grp ? (hasB ? it.y & 1 : it.x & 1) : it.x & 1;
      const int row0 = grp ? SB.row0 : SA.row0;
      const int n = split_n(grp ? SB : SA);
      const int r = 64 * half + 2 * l;
      const bool on = r < n && (grp == 0 || hasB);
      const int i0 = row0 + (r < n ? r : 64 * half);  // idle lanes: the half's first pair
      sb_d2 acc = *(const sb_d2*)(y + i0);
      for (int k0 = 0; k0 < nu; k0 += UCH) {
        int2 ea[UCH], eb[UCH];
#pragma unroll
        for (int k = 0; k < UCH; k++) {
          ea[k] = ul[SA.uoff + k0 + k];
          eb[k] = ul[SB.uoff + k0 + k];
        }
        sb_d2 g[UCH];
        int ix[UCH];
#pragma unroll
        for (int k = 0; k < UCH; k++) {
          const int d = grp ? eb[k].x : ea[k].x;
          ix[k] = grp ? eb[k].y : ea[k].y;
          g[k] = *(const sb_d2*)(x + i0 + d);
        }
        asm volatile("" ::: "memory");  // all gathers in flight before the first use
#pragma unroll
        for (int k = 0; k < UCH; k++) {
          const H h = sdict[ix[k]];
          acc.x = add(acc.x, mul(h, g[k].x));
          acc.y = add(acc.y, mul(h, g[k].y));
        }
      }
      const uint32_t* wp = lw + (grp ? SB.loff : SA.loff) + (i0 - row0);
      for (int k0 = 0; k0 < wl; k0 += kSplitLChunk) {
        sb_u2 c[kSplitLChunk];
        double g0[kSplitLChunk], g1[kSplitLChunk];
#pragma unroll
        for (int k = 0; k < kSplitLChunk; k++) c[k] = ldm<NT>((const sb_u2*)(wp + kSplitRows * (k0 + k)));
#pragma unroll
        for (int k = 0; k < kSplitLChunk; k++) {
          g0[k] = x[c[k].x & kPackColMask];
          g1[k] = x[c[k].y & kPackColMask];
        }
#pragma unroll
        for (int k = 0; k < kSplitLChunk; k++) {
          acc.x = add(acc.x, mul(sdict[c[k].x >> kPackShift], g0[k]));
          acc.y = add(acc.y, mul(sdict[c[k].y >> kPackShift], g1[k]));
        }
      }
      if (on) {
        if constexpr (std::is_same_v<Epi, EpiStore<false>>) {
          __builtin_nontemporal_store(acc, (sb_d2*)(epi.hv + i0));  // one 16-byte store (as pass D)
        } else {
          const sb_d2 xo = *(const sb_d2*)(x + i0);
          part += epi.row((int64_t)i0, acc.x, xo.x);
          part += epi.row((int64_t)i0 + 1, acc.y, xo.y);
        }
      }
    }
    // ---- generic slices (no pair property): one 128-row slice per wavefront
    for (int q = xoffG[xcd] + w0; q < xoffG[xcd + 1]; q += nwx)
      part += sb_generic<HC, VC, NT, UCH>(sl[glist[q]], lane, ul, lw, sdict, x, y, epi);
  } else {
    // ---- complex vectors: one 64-row half per wavefront, one row per lane
    for (int q = xoffI[xcd] + w0; q < xoffI[xcd + 1]; q += nwx) {
      const int e = items[q].x;
      const SplitSlice S = sl[e >> 1];
      const int half = e & 1;
      const int r = 64 * half + lane;
      const bool on = r < split_n(S);
      const int i0 = S.row0 + (on ? r : 64 * half);
      V acc = y[i0];
      for (int k0 = 0; k0 < S.nu; k0 += UCH) {
        int2 ek[UCH];
        V g[UCH];
#pragma unroll
        for (int k = 0; k < UCH; k++) ek[k] = ul[S.uoff + k0 + k];
#pragma unroll
        for (int k = 0; k < UCH; k++) g[k] = x[i0 + ek[k].x];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < UCH; k++) acc = add(acc, mul(sdict[ek[k].y], g[k]));
      }
      const uint32_t* wp = lw + S.loff + (i0 - S.row0);
      for (int k0 = 0; k0 < S.wl; k0 += kSplitLChunk) {
        uint32_t c[kSplitLChunk];
        V g[kSplitLChunk];
#pragma unroll
        for (int k = 0; k < kSplitLChunk; k++) c[k] = ldm<NT>(wp + kSplitRows * (k0 + k));
#pragma unroll
        for (int k = 0; k < kSplitLChunk; k++) g[k] = x[c[k] & kPackColMask];
#pragma unroll
        for (int k = 0; k < kSplitLChunk; k++) acc = add(acc, mul(sdict[c[k] >> kPackShift], g[k]));
      }
      if (on) part += epi.row((int64_t)i0, acc, x[i0]);
    }
  }
  epi.finish(part);
}

}  // namespace edg
