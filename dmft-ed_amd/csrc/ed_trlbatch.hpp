// ed_trlbatch.hpp — thick-restart Lanczos of many small sectors in one launch.
//
// A configs[3] farm has ~70 Lanczos sectors of 495-14,520 rows (ED_DIAG.f90:
// 71-249 loops over them).  Solved one at a time, each Krylov step of such a
// sector is one or more launches of a few microseconds' work: ~18-30 us per
// step of launch chain and latency, and eight farm workers share the four
// hardware queues, so those steps queue behind the large sectors' HBM-bound
// kernels.  Here one workgroup owns one sector for a whole expansion sweep
// (thick-restart rotation, the m - j0 Krylov steps, each an H·v from an LDS
// copy of v_j plus the single-workgroup CGS2 of k_orth_solo), and a launch
// carries every active sector of the batch: one launch and one host round
// trip per restart cycle for all of them.  The host keeps ARPACK's outer
// logic per sector (projected eigenproblem, convergence test, thick restart,
// the degeneracy screen's decisions) exactly as trlan_core / probe_screen
// do, on the numbers the launches leave in a per-sector mailbox.
//
// Per-step arithmetic is that of k_step_solo (stored H, real vectors): the
// H·v row sums in slot order with the shifted three-term epilogue, then
// orth_solo_body (CGS pass 1, local-only or full pass 2, DGKS pass 3,
// alpha/beta, V_{j+1} = w / beta).
#pragma once
#include "ed_trlan.hpp"

namespace edg {

constexpr int kTbBlock = kOrthSoloBlock;  // 512 threads: one workgroup per sector
constexpr int kTbMaxCols = 32;            // orth_solo_body's widest column group
constexpr int kTbMail = 72;               // mailbox: alpha [0, 32) | beta [32, 64) | scalar [64]
constexpr int kTbScreenLen = 416;         // pa / pb entries (kScreenMaxSteps + the norm slot)
constexpr int kTbScreenSlot = kTbScreenLen - 1;
constexpr int64_t kTbMaxDim = 15360;      // v_j staged in LDS (120 KB)
// ed_sectors_eigh_batch gives sectors up to this many rows one workgroup each
// (a workgroup's step grows with the rows: ~13 us at 495-924 rows, ~180 us
// at 14,520) and the larger ones to the lockstep solve
constexpr int64_t kTbWgMaxDim = 2640;

enum : int {
  kTbStart = 0,    // V_0 = w / |w| (w: the uploaded start vector), sweep [0, m)
  kTbRestart = 1,  // V[:, :nrot] = V[:, :ldy] Y, V_nrot = w / beta[m-1], sweep [nrot, m)
  kTbScreen = 2,   // [final rotation,] [screen start,] screen steps [k0s, k1)
};

struct TrlTask {
  // stored H: packed words {col:24 | dict:8} + dictionary, or plain SELL
  const double* diag;
  const int64_t* sptr;
  const uint32_t* words;
  const double* dict;
  const int32_t* cols;
  const double* vals;
  int64_t dim;
  double* Vb;     // basis: column c at Vb + c*dim
  double* w;      // residual
  double* alpha;  // main recurrence alpha[0, 64) | beta[0, 64]; screen pa / pb
  double* beta;
  double* pa;
  double* pb;
  double2* coef;
  double* mail;     // kTbMail doubles the host reads back after the launch
  const double* Y;  // rotation (ldy x nrot, column-major), device
  int op, m, ldy, nrot;
  int nev;          // screen: locked columns [0, nev), window nev, nev + 1
  int k0s, k1;      // screen steps [k0s, k1); k0s == 0: the screen's start vector first
  int hint;         // screen start: + the Ritz vector at column nev (k_mix_hint)
  int locupd;       // local-only CGS update allowed (kCgsLocTol)
  uint64_t seed;    // screen start: hash vector seed (k_hash_vec)
};

__device__ __forceinline__ double tb_hash(int64_t i, uint64_t seed) {  // k_hash_vec's value
  uint64_t z = (uint64_t)(i + 1 + seed * 0x632BE59BD9B4E019ull) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}

// w = H v (v staged in LDS vl, the slice pointers in LDS ssp); shifted:
// w = (H - sg) v - bp vprev.  Row sums in slot order, diagonal first
// (k_step_solo / k_spmv_pk).  Packed words: two rows per iteration, both
// rows' word loads in flight before either row's gathers (one workgroup on
// thousands of rows is bound by the latency of each row's loads).
__device__ __forceinline__ void tb_hxv(const TrlTask& a, const int64_t* ssp, const double* vl, const double* sdict,
                                       double* x, const double* vprev, double sg, double bp, bool shifted) {
  const int t = threadIdx.x;
  const auto diag = gptr(a.diag);
  const auto xg = gptr(x);
  const auto pg = gptr(vprev);
  int64_t i = t;
  if (a.words) {
    const auto wb = gptr(a.words);
    for (; i + kTbBlock < a.dim; i += 2 * kTbBlock) {
      const int64_t j = i + kTbBlock;
      const int64_t s0a = ssp[i >> 6], s0b = ssp[j >> 6];
      const int wa = (int)((ssp[(i >> 6) + 1] - s0a) >> 6), wbn = (int)((ssp[(j >> 6) + 1] - s0b) >> 6);
      const auto pa = wb + s0a + (i & 63);
      const auto pb = wb + s0b + (j & 63);
      const double da = diag[i], db = diag[j];
      const double qa = shifted ? pg[i] : 0.0, qb = shifted ? pg[j] : 0.0;
      const double xa = vl[i], xb = vl[j];
      double acca = 0.0 + da * xa, accb = 0.0 + db * xb;
      const int wm = wa > wbn ? wa : wbn;
      for (int k0 = 0; k0 < wm; k0 += kChunk) {
        uint32_t ca[kChunk], cb[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; k++) {
          ca[k] = (k0 + k < wa) ? pa[64 * (k0 + k)] : 0u;
          cb[k] = (k0 + k < wbn) ? pb[64 * (k0 + k)] : 0u;
        }
#pragma unroll
        for (int k = 0; k < kChunk; k++)
          if (k0 + k < wa) acca = acca + sdict[ca[k] >> kPackShift] * vl[ca[k] & kPackColMask];
#pragma unroll
        for (int k = 0; k < kChunk; k++)
          if (k0 + k < wbn) accb = accb + sdict[cb[k] >> kPackShift] * vl[cb[k] & kPackColMask];
      }
      xg[i] = shifted ? (acca - sg * xa) - bp * qa : acca;
      xg[j] = shifted ? (accb - sg * xb) - bp * qb : accb;
    }
  }
  for (; i < a.dim; i += kTbBlock) {
    const int64_t sl = i >> 6, s0 = ssp[sl];
    const int w = (int)((ssp[sl + 1] - s0) >> 6);
    const double xi = vl[i];
    double acc = 0.0 + diag[i] * xi;
    if (a.words) {
      const auto wp = gptr(a.words) + s0 + (i & 63);
      for (int k0 = 0; k0 < w; k0 += kChunk) {
        uint32_t c[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; k++) c[k] = (k0 + k < w) ? wp[64 * (k0 + k)] : (uint32_t)i;
#pragma unroll
        for (int k = 0; k < kChunk; k++)
          if (k0 + k < w) acc = acc + sdict[c[k] >> kPackShift] * vl[c[k] & kPackColMask];
      }
    } else {
      const auto cp = gptr(a.cols) + s0 + (i & 63);
      const auto hp = gptr(a.vals) + s0 + (i & 63);
      for (int k0 = 0; k0 < w; k0 += kChunk) {
        int32_t c[kChunk];
        double h[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; k++) c[k] = (k0 + k < w) ? cp[64 * (k0 + k)] : (int32_t)i;
#pragma unroll
        for (int k = 0; k < kChunk; k++) h[k] = (k0 + k < w) ? hp[64 * (k0 + k)] : 0.0;
#pragma unroll
        for (int k = 0; k < kChunk; k++)
          if (k0 + k < w) acc = acc + h[k] * vl[c[k]];
      }
    }
    xg[i] = shifted ? (acc - sg * xi) - bp * pg[i] : acc;
  }
}

// V[:, :nout] = V[:, :ncol] Y (Y ncol x nout, column-major, in LDS), in
// place row by row (k_rotate_ip's order); with scale_col >= 0 also
// V[:, scale_col] = w * inv
template <int NC>
__device__ __forceinline__ void tb_rotate(double* Vb, int64_t dim, const double* ys, int ncol, int nout,
                                          const double* w, int scale_col, double inv) {
  const auto Vg = gptr(Vb);
  const auto wg = gptr(w);
  for (int64_t i = threadIdx.x; i < dim; i += kTbBlock) {
    double v[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) v[c] = c < ncol ? Vg[(int64_t)c * dim + i] : 0.0;
    for (int k = 0; k < nout; k++) {
      double acc = 0.0;
#pragma unroll
      for (int c = 0; c < NC; c++)
        if (c < ncol) acc = acc + ys[c + k * ncol] * v[c];
      Vg[(int64_t)k * dim + i] = acc;
    }
    if (scale_col >= 0) Vg[(int64_t)scale_col * dim + i] = inv * wg[i];
  }
}

// block sum of x^2 in a fixed order (every thread gets it)
__device__ __forceinline__ double tb_norm2(const double* x, int64_t dim) {
  __shared__ double red[kTbBlock / 64];
  double s = 0.0;
  const auto xg = gptr(x);
  for (int64_t i = threadIdx.x; i < dim; i += kTbBlock) s += xg[i] * xg[i];
  s = wave_sum_dpp(s);
  if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = s;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int k = 0; k < kTbBlock / 64; k++) r = r + red[k];
  __syncthreads();
  return r;
}

// One instantiation per column bound NC (24: Nblock <= 24, else 32): the
// sweep's column groups all use NC registers (loads stay guarded by ncol), so
// the kernel holds one orth_solo_body, not four (four inlined: 1,318 SGPR
// spills).
template <int NC>
__global__ void __launch_bounds__(kTbBlock) k_trl_batch(const TrlTask* __restrict__ tasks) {
  extern __shared__ double vl[];  // v_j of the current step (dim doubles)
  __shared__ double sdict[256];
  __shared__ double ys[kTbMaxCols * kTbMaxCols];
  __shared__ int64_t ssp[kTbMaxDim / 64 + 2];  // SELL slice pointers
  const TrlTask a = tasks[blockIdx.x];
  const int t = threadIdx.x;
  const int64_t dim = a.dim;
  auto col = [&](int c) { return a.Vb + (int64_t)c * dim; };
  if (a.words && t < 256) sdict[t] = a.dict[t];
  for (int64_t k = t; k <= (dim + 63) / 64; k += kTbBlock) ssp[k] = a.sptr[k];
  if (a.nrot > 0)
    for (int k = t; k < a.ldy * a.nrot; k += kTbBlock) ys[k] = a.Y[k];
  __syncthreads();
  // one Krylov step: stage v (column vc), w = H v [shifted], CGS2 + alpha/beta, out
  auto step = [&](int vc, int pc, const double* al, const double* be, int kprev, bool shifted, int ncol,
                  double* alpha, double* beta, int jn, double* out, int jc) {
    __syncthreads();  // previous step's out / alpha / beta written
    const auto v = gptr(col(vc));
#pragma unroll 4
    for (int64_t i = t; i < dim; i += kTbBlock) vl[i] = v[i];
    const double sg = shifted ? al[kprev] : 0.0, bp = shifted ? be[kprev] : 0.0;
    __syncthreads();
    tb_hxv(a, ssp, vl, sdict, a.w, shifted ? col(pc) : nullptr, sg, bp, shifted);
    // (the CGS passes read back only each thread's own rows of w)
    orth_solo_body<false, NC, (NC <= 24 ? 2 : 1)>(a.Vb, ncol, a.w, dim, a.coef, alpha, beta, jn, jn, out, shifted ? 1 : 0,
            (shifted && a.locupd) ? 1 : 0, jc);
  };
  if (a.op == kTbStart || a.op == kTbRestart) {
    int j0 = 0;
    if (a.op == kTbStart) {
      const double b0 = sqrt(tb_norm2(a.w, dim));
      const double inv = b0 > 0.0 ? 1.0 / b0 : 0.0;
      for (int64_t i = t; i < dim; i += kTbBlock) a.Vb[i] = inv * a.w[i];
      if (t == 0) a.mail[64] = b0;
    } else {
      const double bm = a.beta[a.m - 1];
      tb_rotate<NC>(a.Vb, dim, ys, a.ldy, a.nrot, a.w, a.nrot, bm > 0.0 ? 1.0 / bm : 0.0);
      j0 = a.nrot;
    }
    for (int j = j0; j < a.m; j++) {
      const bool sh = j > j0;
      step(j, j - 1, a.alpha, a.beta, j - 1, sh, j + 1, a.alpha, a.beta, j, j + 1 < a.m ? col(j + 1) : nullptr, -1);
    }
    __syncthreads();
    if (t < a.m) {
      a.mail[t] = a.alpha[t];
      a.mail[32 + t] = a.beta[t];
    }
    return;
  }
  // degeneracy screen (probe_screen): rolling window ca / cb behind the
  // nev locked columns, alpha / beta in pa / pb
  const int ca = a.nev, cb = a.nev + 1;
  if (a.nrot > 0) {  // Ritz vectors of the main solve -> V[:, :nrot]
    tb_rotate<NC>(a.Vb, dim, ys, a.ldy, a.nrot, nullptr, -1, 0.0);
    __syncthreads();
  }
  if (a.k0s == 0 && a.k1 > 0) {
    const double amix = sqrt((double)dim / 3.0);
    for (int64_t i = t; i < dim; i += kTbBlock) {
      double h = tb_hash(i, a.seed);
      if (a.hint) h = h + amix * col(ca)[i];
      a.w[i] = h;
      col(cb)[i] = 0.0;  // v_{-1} = 0
    }
    __syncthreads();
    // against the locked columns; the norm -> pb[kScreenMaxSteps + 1]; v_0 -> column ca
    orth_solo_body<false, NC, (NC <= 24 ? 2 : 1)>(a.Vb, a.nev, a.w, dim, a.coef, nullptr, a.pb, -1, kTbScreenSlot, col(ca), 0, 0);
  }
  for (int k = a.k0s; k < a.k1; k++) {
    const int cur = (k & 1) ? cb : ca, prv = (k & 1) ? ca : cb;
    step(cur, prv, a.pa, a.pb, k - 1, k > 0, a.nev + 2, a.pa, a.pb, k, col(prv), cur);
  }
  __syncthreads();
  const int n = a.k1 - a.k0s;
  if (t < n) {
    a.mail[t] = a.pa[a.k0s + t];
    a.mail[32 + t] = a.pb[a.k0s + t];
  }
  if (t == 0) a.mail[64] = a.pb[kTbScreenSlot];
}

}  // namespace edg
