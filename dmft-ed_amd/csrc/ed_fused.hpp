// ed_fused.hpp — one-pass stored H·v on a re-laid matrix (round 6).
//
// spMatVec_cc (ED_HAMILTONIAN_STORED_HxV.f90:132-143) streams one word per
// stored element.  The cross-block elements of a 64-row unit of one idw block
// (the down-spin hops of normal and nonSU2 sectors: target (idw', same up
// rank), same Jordan-Wigner sign, same value on every row of the unit) are
// the same {column offset, value} for all 64 rows; the two-segment form
// (ed_split.hpp) stores them once per slice as U entries but pays a second
// sweep and a y round trip, which complex(8) vectors cannot keep in the 256 MB
// Infinity Cache (v and y are 188 MB each at Nlevels=28).  This form keeps
// the U compression and the single row-order sweep:
//
//   unit = <= 64 consecutive rows of one idw block (one wavefront, one row
//   per lane), in row order, one contiguous eighth of the units per XCD;
//   A words: the in-block elements {col:24 | dictionary index:8}, slot-major
//     (word k of lane l at aoff + 64 k + l), insertion order;
//   U list:  the cross-block elements every row of the unit holds with the
//     same {col - row, dictionary index}: one wave-uniform scalar load and one
//     coalesced gather (512 B real, 1 KB complex) per element;
//   L words: the remaining cross-block elements (spin flips, Jx/Jp, pair
//     terms), per lane like the A words.
//
// The re-lay is lossless (every stored element once, the stored value), built
// on the device from the packed SELL words.  Summation order: diagonal, the
// in-block elements in insertion order, U, L — the order of the two-segment
// form (a reordering of spMatVec_cc's row sum: 1e-13 of the row's |H||x|,
// tests/test_gpu_fused.py; ED_OPT_STORED_EXACT keeps the bit-identical
// one-pass kernel).  Real and complex H (complex dictionary of (re, im)
// pairs), real and complex vectors.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ed_kernels.hpp"

namespace edg {

struct FuUnit {
  int32_t row0;   // first row
  int32_t n;      // rows (<= 64)
  int32_t wa;     // A words per row (slots)
  int32_t nu;     // U entries, padded to kFuUChunk with {0, zero value}
  int32_t wl;     // L words per row, padded to kFuLChunk
  int32_t pad_;
  int64_t aoff;   // first A word (64 * wa words, slot-major)
  int64_t uoff;   // first U entry
  int64_t loff;   // first L word (64 * wl words, slot-major)
};
constexpr int kFuFarMax = 32;    // cross-block elements per row the build stages
constexpr int kFuUChunk = 8;     // U entries per load batch (lists padded to it, or to 7)
#ifndef ED_FU_LCH
#define ED_FU_LCH 4
#endif
#ifndef ED_FU_CHMAX
#define ED_FU_CHMAX 8
#endif
constexpr int kFuLChunk = ED_FU_LCH;  // L slots per load batch
// widest A batch: rows of up to 12 in-block elements (Norb=2) take a batch of
// 8 and one of 4 rather than one of 12 — complex vectors on real H 0.37 ->
// 0.30 ms at N28b, 0.42 -> 0.33 at N28 with Jx/Jp, real vectors -4 %
// (gpurun_out r6c, A/B builds -DED_FU_CHMAX=16 / 8)
constexpr int kFuChMax = ED_FU_CHMAX;
constexpr int kFuBuildBlock = 256;  // 4 waves: 4 x 32 x 64 keys of 8 B = 64 KB of LDS

// ---- build: one wavefront per unit, one row per lane.  FILL = false: the
// unit's A width, U count, L width (and the largest cross-block count of any
// row, atomicMax into *farmax); FILL = true: A words, U list and L words at
// the unit's offsets.  Each row's cross-block elements are staged in LDS as
// 64-bit keys {col - row : 32 | dictionary index : 32}; an element of the
// unit's first row is uniform when every row holds the same key (matched
// against the first not yet matched occurrence: duplicate keys in a row are
// matched once each).
template <bool FILL>
__global__ void __launch_bounds__(kFuBuildBlock) k_fu_build(const int64_t* __restrict__ sptr,
                                                            const uint32_t* __restrict__ words,
                                                            const uint16_t* __restrict__ cnt,
                                                            const uint32_t* __restrict__ map, int ns,
                                                            FuUnit* __restrict__ units, int64_t nunit,
                                                            uint32_t* __restrict__ wa, int2* __restrict__ ul,
                                                            uint32_t* __restrict__ lw, uint32_t zpad, int* farmax,
                                                            unsigned long long* nfar) {
  constexpr int NW = kFuBuildBlock / 64;
  __shared__ unsigned long long keys[NW][kFuFarMax][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int64_t q = (int64_t)blockIdx.x * NW + wv; q < nunit; q += (int64_t)gridDim.x * NW) {
    const int64_t qq = __builtin_amdgcn_readfirstlane((int)q);
    const FuUnit U = units[qq];
    const bool on = lane < U.n;
    const int64_t i = U.row0 + (on ? lane : 0);
    const uint32_t blk = map[i] >> ns;
    const uint32_t* wp = words + sptr[i >> 6] + (i & 63);
    const int c = on ? cnt[i] : 0;
    int na = 0, nf = 0;
    for (int k = 0; k < c; k++) {
      const uint32_t wd = wp[64 * k];
      const uint32_t col = wd & kPackColMask;
      if ((map[col] >> ns) == blk) {
        if constexpr (FILL) wa[U.aoff + 64 * (int64_t)na + lane] = wd;
        na++;
      } else {
        if (nf < kFuFarMax)
          keys[wv][nf][lane] = ((unsigned long long)(uint32_t)((int32_t)col - (int32_t)i) << 32) | (wd >> kPackShift);
        nf++;
      }
    }
    const int nfs = min(nf, kFuFarMax);
    const int nf0 = __builtin_amdgcn_readfirstlane(nfs);  // lane 0 (row0) always holds a row
    uint32_t used = 0u;
    int nuu = 0;
    for (int k0 = 0; k0 < nf0; k0++) {
      const unsigned long long key = keys[wv][k0][0];
      int pos = -1;
      for (int j = nfs - 1; j >= 0; j--)
        if (!((used >> j) & 1u) && keys[wv][j][lane] == key) pos = j;
      const bool mine = !on || pos >= 0;
      if (__ballot(mine) == __ballot(1)) {
        if (on) used |= 1u << pos;
        if constexpr (FILL) {
          if (lane == 0) ul[U.uoff + nuu] = make_int2((int32_t)(key >> 32), (int32_t)(key & 0xffu));
        }
        nuu++;
      }
    }
    const int nl = on ? nfs - __popc(used) : 0;
    if constexpr (!FILL) {
      const int wmax = wave_max(na), lmax = wave_max(nl), fmax = wave_max(nf);
      const double sfar = wave_sum((double)nf);
      if (lane == 0) {
        units[qq].wa = wmax;
        units[qq].nu = nuu;
        units[qq].wl = lmax;
        atomicMax(farmax, fmax);
        atomicAdd(nfar, (unsigned long long)sfar);
      }
    } else {
      // padding: own column, the dictionary's zero
      const uint32_t pad = (uint32_t)i | zpad;
      for (int k = na; k < U.wa; k++) wa[U.aoff + 64 * (int64_t)k + lane] = pad;
      for (int k = nuu + lane; k < U.nu; k += 64) ul[U.uoff + k] = make_int2(0, (int32_t)(zpad >> kPackShift));
      int k2 = 0;
      for (int j = 0; j < nfs; j++)
        if (!((used >> j) & 1u)) {
          const unsigned long long kk = keys[wv][j][lane];
          lw[U.loff + 64 * (int64_t)(k2++) + lane] =
              (uint32_t)((int32_t)i + (int32_t)(kk >> 32)) | ((uint32_t)(kk & 0xffu) << kPackShift);
        }
      for (; k2 < U.wl; k2++) lw[U.loff + 64 * (int64_t)k2 + lane] = pad;
    }
  }
}

// ---- H·v: one wavefront per unit (row per lane), units in row order, XCD x
// walking the x-th eighth of the list (its L2 serves the in-block gathers of
// a block's consecutive units and the cross-block gathers its neighbouring
// rows share).  Every load of a batch is issued before the first is used.
// CH: A slots per batch; UCH: U entries per batch (the lists are padded to it).
template <bool HC, bool VC, int NT, class Epi, int CH, int UCH>
__global__ void __launch_bounds__(kBlock) k_spmv_fu(const val_t<HC>* __restrict__ diag,
                                                    const FuUnit* __restrict__ units, int64_t nunit,
                                                    const uint32_t* __restrict__ wa, const int2* __restrict__ ul,
                                                    const uint32_t* __restrict__ lw,
                                                    const val_t<HC>* __restrict__ dict,
                                                    const val_t<VC>* __restrict__ x, Epi epi) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  if (epi.skip()) return;
  epi.prepare();
  __shared__ H sdict[256];
  sdict[threadIdx.x] = dict[threadIdx.x];  // kBlock == 256 == dictionary capacity
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int xcd = blockIdx.x & 7;
  const int64_t q_lo = nunit * xcd / 8, q_hi = nunit * (xcd + 1) / 8;
  const int64_t nwx = (int64_t)(gridDim.x >> 3) * (kBlock / 64);  // waves per XCD
  double part = 0.0;
  for (int64_t q = q_lo + (int64_t)(blockIdx.x >> 3) * (kBlock / 64) + wv; q < q_hi; q += nwx) {
    const FuUnit U = units[q];
    const bool on = lane < U.n;
    const int64_t i = U.row0 + (on ? lane : 0);
    const V xi = x[i];
    const H dg = ldh<NT>(diag + i);
    V acc = mul(dg, xi);
    // A: in-block elements (branch-free batches: slots past the width reload
    // the last slot and are dropped by a select)
    if (U.wa > 0) {
      const uint32_t* ap = wa + U.aoff + lane;
      const int wm = U.wa - 1;
      for (int k0 = 0; k0 < U.wa; k0 += CH) {
        uint32_t c[CH];
#pragma unroll
        for (int k = 0; k < CH; k++) c[k] = ldm<NT>(ap + 64 * min(k0 + k, wm));
        V g[CH];
        H h[CH];
#pragma unroll
        for (int k = 0; k < CH; k++) {
          g[k] = x[c[k] & kPackColMask];
          h[k] = sdict[c[k] >> kPackShift];
        }
        asm volatile("" ::: "memory");  // every gather in flight before the first use
#pragma unroll
        for (int k = 0; k < CH; k++) acc = sel(k0 + k < U.wa, add(acc, mul(h[k], g[k])), acc);
      }
    }
    // U: unit-uniform cross-block elements (padded list: whole batches)
    for (int k0 = 0; k0 < U.nu; k0 += UCH) {
      int2 e[UCH];
#pragma unroll
      for (int k = 0; k < UCH; k++) e[k] = ul[U.uoff + k0 + k];
      V g[UCH];
#pragma unroll
      for (int k = 0; k < UCH; k++) g[k] = x[i + e[k].x];
      asm volatile("" ::: "memory");
#pragma unroll
      for (int k = 0; k < UCH; k++) acc = add(acc, mul(sdict[e[k].y], g[k]));
    }
    // L: the remaining cross-block elements, per lane
    if (U.wl > 0) {
      const uint32_t* lp = lw + U.loff + lane;
      for (int k0 = 0; k0 < U.wl; k0 += kFuLChunk) {
        uint32_t c[kFuLChunk];
#pragma unroll
        for (int k = 0; k < kFuLChunk; k++) c[k] = ldm<NT>(lp + 64 * (k0 + k));
        V g[kFuLChunk];
#pragma unroll
        for (int k = 0; k < kFuLChunk; k++) g[k] = x[c[k] & kPackColMask];
        asm volatile("" ::: "memory");
#pragma unroll
        for (int k = 0; k < kFuLChunk; k++) acc = add(acc, mul(sdict[c[k] >> kPackShift], g[k]));
      }
    }
    if (on) part += epi.row(i, acc, xi);
  }
  epi.finish(part);
}

}  // namespace edg
