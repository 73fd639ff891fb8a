// ed_trlmulti.hpp — thick-restart Lanczos of many stored sectors in lockstep.
//
// One sector's Krylov step is 7 dependent launches (H·v, three CGS passes,
// two coefficient sums, alpha/beta + V_{j+1}); in the configs[3] farm eight
// such chains share the device's four hardware queues, and the queues run
// mostly small kernels one after the other: the 101 sectors above 2,640 rows
// stream ~1.6 TB in ~0.55 s, ~3 TB/s.  Here every kernel of a step carries
// the same step of ALL sectors still running (a flattened grid: each sector
// owns a contiguous block range, found by a binary search over the block
// offsets), so a step is 7 launches for the whole farm and each launch is
// as wide as the sum of the sectors' grids.  The per-sector arithmetic is
// Trlan::step/orth's multi-kernel path (ed_lib.hip) on each sector's own
// grid G: the same CGS passes (cgs_body), coefficient sums (k_vdot_fin's
// order), DGKS and local-only decisions, alpha/beta and V_{j+1}; the host
// runs trlan_core's / probe_screen's per-sector logic on the mailboxes
// (tb_advance, shared with the one-workgroup batch of ed_trlbatch.hpp).
#pragma once
#include "ed_trlbatch.hpp"

namespace edg {

constexpr int kTmFinBlocks = 32;  // coefficient blocks per sector (one per basis column)
constexpr int kTmRowsPerBlock = 2048;  // rows per block of the CGS / coefficient / rotation sweeps
constexpr int kTmMaxEntries = kBlock;  // sectors per lockstep solve (tm_entry)

struct TmSec {  // per sector, fixed for the call
  const double* diag;
  const int64_t* sptr;
  const uint32_t* words;
  const double* dict;
  int64_t dim;
  double* Vb;
  double* w;
  double2* part;   // CGS pass 1 partials (kTrlanMaxCols x G)
  double2* part2;  // pass 2
  double* npA;     // |w|^2 partials before / after the first pass, after the last
  double* npB;
  double* npart;
  double2* h;
  double2* coef;
  int* lof;
  double* alpha;  // main recurrence (72) | beta (72)
  double* beta;
  double* pa;  // screen recurrence (kTbScreenLen each)
  double* pb;
  double* mail;  // kTbMail
  int G;         // blocks of the CGS / coefficient / rotation sweeps
  int Gh;        // blocks of the H·v
};

struct TmCyc {  // per running sector, this cycle
  int sec;        // TmSec index
  int phase;      // 0: main sweep j0..m-1; 1: screen (start when sstart, steps k0s..k1-1)
  int j0, m;
  int k0s, k1, nev, sstart, hint;
  int nrot, ldy, scale_col;  // rotation before the steps
  int locupd;
  uint64_t seed;
  const double* Y;
};

// Sector entry of a flattened block index (boff: n + 1 ascending offsets,
// n <= kBlock): every thread tests one entry's range (two loads in
// parallel, one barrier) instead of a chain of dependent scalar loads
__device__ __forceinline__ int tm_entry(const int* __restrict__ boff, int n, int b) {
  __shared__ int es;
  const int t = threadIdx.x;
  if (t < n && boff[t] <= b && b < boff[t + 1]) es = t;
  __syncthreads();
  return es;
}

struct TmStep {
  bool on, start, shifted;
  int xc, pc, ncol, slot, outc, jc;
  double* al;  // alpha slots (null: none written)
  double* be;
};

// The step `step` of one entry: main j = j0 + step; screen: step 0 is the
// start (hash + hint, CGS against the locked columns, V_ca = w / |w|) when
// sstart, then k = k0s + ... on the rolling window ca / cb.
__device__ __forceinline__ TmStep tm_step(const TmCyc& c, const TmSec& s, int step) {
  TmStep p{};
  if (c.phase == 0) {
    const int j = c.j0 + step;
    p.on = j < c.m;
    p.xc = j;
    p.pc = j - 1;
    p.shifted = j > c.j0;
    p.ncol = j + 1;
    p.slot = j;
    p.outc = j + 1 < c.m ? j + 1 : -1;
    p.jc = j;
    p.al = s.alpha;
    p.be = s.beta;
    return p;
  }
  const int ca = c.nev, cb = c.nev + 1;
  if (c.sstart && step == 0) {
    p.on = c.k1 > c.k0s;
    p.start = true;
    p.ncol = c.nev;
    p.slot = kTbScreenSlot;
    p.outc = ca;
    p.jc = -1;
    p.be = s.pb;
    return p;
  }
  const int k = c.k0s + step - (c.sstart ? 1 : 0);
  p.on = k < c.k1;
  p.xc = (k & 1) ? cb : ca;
  p.pc = (k & 1) ? ca : cb;
  p.shifted = k > 0;
  p.ncol = c.nev + 2;
  p.slot = k;
  p.outc = p.pc;
  p.jc = p.xc;
  p.al = s.pa;
  p.be = s.pb;
  return p;
}

// Rotation before the steps: V[:, :nrot] = V[:, :ldy] Y (in place per row,
// k_rotate_ip's order); scale_col >= 0: V[:, scale_col] = w / beta[m-1]
// (the thick restart's residual column)
__global__ void __launch_bounds__(kBlock) k_tm_rotate(const TmSec* __restrict__ secs, const TmCyc* __restrict__ cyc,
                                                      const int* __restrict__ boff, int n) {
  __shared__ double ys[kTbMaxCols * kTbMaxCols];
  const int e = tm_entry(boff, n, blockIdx.x);
  const TmCyc c = cyc[e];
  if (c.nrot <= 0 && c.scale_col < 0) return;
  const TmSec s = secs[c.sec];
  const int bx = blockIdx.x - boff[e];
  for (int k = threadIdx.x; k < c.ldy * c.nrot; k += kBlock) ys[k] = c.Y[k];
  __syncthreads();
  const double bm = c.scale_col >= 0 ? s.beta[c.m - 1] : 0.0;
  const double inv = bm > 0.0 ? 1.0 / bm : 0.0;
  for (int64_t i = (int64_t)bx * kBlock + threadIdx.x; i < s.dim; i += (int64_t)s.G * kBlock) {
    double v[kTbMaxCols];
#pragma unroll
    for (int q = 0; q < kTbMaxCols; q++) v[q] = q < c.ldy && c.nrot > 0 ? s.Vb[(int64_t)q * s.dim + i] : 0.0;
    for (int k = 0; k < c.nrot; k++) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < kTbMaxCols; q++)
        if (q < c.ldy) acc = acc + ys[q + k * c.ldy] * v[q];
      s.Vb[(int64_t)k * s.dim + i] = acc;
    }
    if (c.scale_col >= 0) s.Vb[(int64_t)c.scale_col * s.dim + i] = inv * s.w[i];
  }
}

// w = H V_xc (packed stored rows, k_spmv_pk's per-row sum: diagonal, then
// the slots in order) with EpiTrlLoc's shifted epilogue; the screen's start
// step writes w = hash + hint instead (k_hash_vec + k_mix_hint) and V_cb = 0
__global__ void __launch_bounds__(kBlock) k_tm_hxv(const TmSec* __restrict__ secs, const TmCyc* __restrict__ cyc,
                                                   const int* __restrict__ boff, int n, int step) {
  __shared__ double sdict[256];
  const int e = tm_entry(boff, n, blockIdx.x);
  const TmCyc c = cyc[e];
  const TmSec s = secs[c.sec];
  const TmStep p = tm_step(c, s, step);
  if (!p.on) return;
  const int bx = blockIdx.x - boff[e];
  const int64_t dim = s.dim;
  if (p.start) {
    const double amix = sqrt((double)dim / 3.0);
    const double* hv = s.Vb + (int64_t)c.nev * dim;
    double* vcb = s.Vb + (int64_t)(c.nev + 1) * dim;
    for (int64_t i = (int64_t)bx * kBlock + threadIdx.x; i < dim; i += (int64_t)s.Gh * kBlock) {
      double h = tb_hash(i, c.seed);
      if (c.hint) h = h + amix * hv[i];
      s.w[i] = h;
      vcb[i] = 0.0;
    }
    return;
  }
  if (threadIdx.x < 256) sdict[threadIdx.x] = s.dict[threadIdx.x];
  __syncthreads();
  const double* x = s.Vb + (int64_t)p.xc * dim;
  const double* vprev = s.Vb + (int64_t)p.pc * dim;
  const double sg = p.shifted ? p.al[p.slot - 1] : 0.0, bp = p.shifted ? p.be[p.slot - 1] : 0.0;
  for (int64_t i = (int64_t)bx * kBlock + threadIdx.x; i < dim; i += (int64_t)s.Gh * kBlock) {
    const int64_t sl = i >> 6, s0 = s.sptr[sl];
    const int w = (int)((s.sptr[sl + 1] - s0) >> 6);
    const uint32_t* wp = s.words + s0 + (i & 63);
    const double xi = x[i];
    double acc = 0.0 + s.diag[i] * xi;
    for (int k0 = 0; k0 < w; k0 += kChunk) {
      uint32_t cw[kChunk];
#pragma unroll
      for (int k = 0; k < kChunk; k++) cw[k] = (k0 + k < w) ? wp[64 * (k0 + k)] : (uint32_t)i;
      double g[kChunk];
#pragma unroll
      for (int k = 0; k < kChunk; k++) g[k] = x[cw[k] & kPackColMask];
#pragma unroll
      for (int k = 0; k < kChunk; k++)
        if (k0 + k < w) acc = acc + sdict[cw[k] >> kPackShift] * g[k];
    }
    s.w[i] = p.shifted ? (acc - sg * xi) - bp * vprev[i] : acc;
  }
}

// One CGS pass of the step on every entry (Trlan::orth's three fused sweeps):
// pass 1 dots + |w|^2; pass 2 w -= V h (local-only decision) + dots +
// |w'|^2; pass 3 the DGKS-conditional second update + |w''|^2
template <int NC>
__global__ void __launch_bounds__(kBlock) k_tm_cgs(const TmSec* __restrict__ secs, const TmCyc* __restrict__ cyc,
                                                   const int* __restrict__ boff, int n, int step, int pass) {
  const int e = tm_entry(boff, n, blockIdx.x);
  const TmCyc c = cyc[e];
  const TmSec s = secs[c.sec];
  const TmStep p = tm_step(c, s, step);
  if (!p.on) return;
  const int bx = blockIdx.x - boff[e];
  const bool lf = p.shifted && c.locupd;
  if (pass == 1)
    cgs_body<false, NC>(s.Vb, p.ncol, nullptr, s.w, s.dim, s.part, s.npA, nullptr, 0, nullptr, 0, nullptr, nullptr,
                        nullptr, nullptr, s.G, bx);
  else if (pass == 2)
    cgs_body<false, NC>(s.Vb, p.ncol, s.h, s.w, s.dim, s.part2, s.npB, nullptr, 0, nullptr, 0, nullptr, nullptr,
                        lf ? s.lof : nullptr, lf ? s.npA : nullptr, s.G, bx);
  else
    cgs_body<false, NC>(s.Vb, p.ncol, s.h, s.w, s.dim, nullptr, s.npart, nullptr, 0, nullptr, 0, s.npA, s.npB,
                        lf ? s.lof : nullptr, nullptr, s.G, bx);
}

// The pass's coefficients h[c] = sum_b part[c*G + b] (k_vdot_fin); pass 1
// sets coef = h, pass 2 adds (skipped with the DGKS test, like k_vdot_fin)
__global__ void __launch_bounds__(kBlock) k_tm_fin(const TmSec* __restrict__ secs, const TmCyc* __restrict__ cyc,
                                                   int n, int step, int pass) {
  const int e = blockIdx.x / kTmFinBlocks, cc = blockIdx.x % kTmFinBlocks;
  const TmCyc c = cyc[e];
  const TmSec s = secs[c.sec];
  const TmStep p = tm_step(c, s, step);
  if (!p.on || cc >= p.ncol) return;
  const double2* part = pass == 1 ? s.part : s.part2;
  if (pass == 2 && dgks_skip(s.npA, s.npB, s.G)) return;
  double re = 0.0;
  for (int b = threadIdx.x; b < s.G; b += kBlock) re += part[(int64_t)cc * s.G + b].x;
  re = block_sum(re);
  if (threadIdx.x == 0) {
    s.h[cc] = make_double2(re, 0.0);
    if (pass == 2) s.coef[cc] = make_double2(s.coef[cc].x + re, s.coef[cc].y);
    else s.coef[cc] = make_double2(re, 0.0);
  }
}

// beta[slot] = |w|, alpha[slot] (shifted: alpha[slot-1] + <v, w>), and
// V_outc = w / beta (k_coef_scale / k_trl_coef)
__global__ void __launch_bounds__(kBlock) k_tm_coef(const TmSec* __restrict__ secs, const TmCyc* __restrict__ cyc,
                                                    const int* __restrict__ boff, int n, int step) {
  const int e = tm_entry(boff, n, blockIdx.x);
  const TmCyc c = cyc[e];
  const TmSec s = secs[c.sec];
  const TmStep p = tm_step(c, s, step);
  if (!p.on) return;
  const int bx = blockIdx.x - boff[e];
  double t = 0.0;
  for (int b = threadIdx.x; b < s.G; b += kBlock) t += s.npart[b];
  t = block_sum(t);
  const double nrm = sqrt(t);
  if (bx == 0 && threadIdx.x == 0) {
    p.be[p.slot] = nrm;
    if (p.al) p.al[p.slot] = p.shifted ? p.al[p.slot - 1] + s.coef[p.jc].x : s.coef[p.jc].x;
  }
  if (p.outc < 0) return;
  const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;
  double* out = s.Vb + (int64_t)p.outc * s.dim;
  for (int64_t i = (int64_t)bx * kBlock + threadIdx.x; i < s.dim; i += (int64_t)s.G * kBlock) out[i] = inv * s.w[i];
}

// Mailbox of the cycle (one block per entry): main alpha/beta [0, m), screen
// pa/pb [k0s, k1), slot 64 the screen start's norm (1 on the main path)
__global__ void __launch_bounds__(64) k_tm_mail(const TmSec* __restrict__ secs, const TmCyc* __restrict__ cyc) {
  const TmCyc c = cyc[blockIdx.x];
  const TmSec s = secs[c.sec];
  const int t = threadIdx.x;
  if (c.phase == 0) {
    if (t < c.m) {
      s.mail[t] = s.alpha[t];
      s.mail[32 + t] = s.beta[t];
    }
    if (t == 0) s.mail[64] = 1.0;
  } else {
    if (t < c.k1 - c.k0s) {
      s.mail[t] = s.pa[c.k0s + t];
      s.mail[32 + t] = s.pb[c.k0s + t];
    }
    if (t == 0) s.mail[64] = s.pb[kTbScreenSlot];
  }
}

}  // namespace edg
