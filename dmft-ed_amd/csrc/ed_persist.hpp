// ed_persist.hpp — one-workgroup persistent Lanczos for small sectors.
//
// For sectors whose Lanczos vector fits in LDS (configs[1]: dim 4,900 real =
// 39 KB) the per-iteration cost of the multi-kernel recurrence is launch and
// grid-reduction latency, not bandwidth (≈10 µs per iteration for 4,900 rows).
// Here one 1024-thread workgroup (16 wavefronts, one CU) runs many
// iterations of the .repo/PLAIN_LANCZOS.f90:87-118 recurrence without leaving
// the CU:
//   * v (the current normalised Lanczos vector) lives in LDS and is gathered
//     by the H·v; p = v_{k-1} and w live in registers of the thread that owns
//     the row (row i = tid + r*1024, r < RPT);
//   * H is the stored SELL-64 matrix streamed from L2 (MODE 0, same element
//     order as k_spmv -> same H·v bits), the Kronecker tables copied into
//     LDS (MODE 1, normal mode without Jx/Jp), or the stored matrix held in
//     REGISTERS (MODE 2, ELL layout): row i = tid + r*NT keeps its W
//     off-diagonal entries as 32-bit words {col:17 | value byte offset:14}
//     into a dictionary of the distinct values (hoppings/exchange: a few
//     dozen), padded with the dictionary's 0.0; diagonal, dictionary and v in
//     LDS.  No matrix byte leaves the CU after the first iteration and the
//     entry loop has no branch, so every gather of a row is in flight at once;
//     MODE 3 is the matrix-free twin: the same words generated in-kernel
//     from the Kronecker hop tables (dictionary = the tables' values);
//   * alpha and beta are block reductions (wave shuffles + 16-entry LDS),
//     three barriers per iteration, no global synchronisation.
// Independent runs (GF seeds, sector replicas) use one workgroup each
// (blockIdx.x indexes PersistRun[]), so up to 256 chains run side by side.
#pragma once
#include "ed_kernels.hpp"

namespace edg {

constexpr int kPBlock = 1024;
constexpr int kPChunk = 8;
constexpr int kPRegBlock = 512;  // MODE 2 block: 256-VGPR lanes hold the packed matrix

template <bool HC>
struct PersistRun {
  using H = val_t<HC>;
  // stored matrix (MODE 0)
  const H* diag;
  const int64_t* sptr;
  const int32_t* cols;
  const H* vals;
  // Kronecker tables (MODE 1)
  KronArgs<HC> K;
  int64_t dim;
  void* R;           // in: start vector (first) or saved v; out: saved v
  void* P;           // saved p
  LancState* st;     // beta, iter, done, thresh
  double* alpha;     // [niter_total]
  double* beta;      // [niter_total+1]
  void* basis;       // optional Krylov basis (column k = v_k), or null
  // register-resident stored matrix (MODE 2)
  const uint32_t* pk;   // [RPT*W][kPRegBlock] packed entries
  const H* dict;        // [ndict] distinct values, dict[0] = 0
  int ndict;
  int niter;         // iterations in this launch
  int first;         // 1: R holds the unnormalised start vector
};

// TAIL=false drops the trailing barrier: the caller guarantees a barrier
// between this read of ws and the next write to the same buffer (the
// iteration alternates two buffers, separated by the step's barriers).
template <int NT = kPBlock, bool TAIL = true>
__device__ __forceinline__ double pblock_sum(double v, double* ws) {
  v = wave_sum(v);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) ws[wv] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) t = t + ws[w];
  if constexpr (TAIL) __syncthreads();
  return t;
}

constexpr uint32_t kPkColBits = 17, kPkColMask = (1u << kPkColBits) - 1;
constexpr uint32_t kPkOffMask = (1u << 14) - 1;  // dictionary byte offset (<= 16 KiB)

template <bool HC, bool VC, int MODE, int RPT, int E = 1, int NT = kPBlock>
__global__ void __launch_bounds__(NT) k_lanc_persist(const PersistRun<HC>* __restrict__ runs) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  const PersistRun<HC>& a = runs[blockIdx.x];  // uniform: scalar loads, no VGPR copy
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ double ws[NT / 64];
  __shared__ double ws2[NT / 64];  // beta's buffer: alpha/beta alternate, one barrier each
  V* vl = (V*)smem;  // MODE 2 moves it behind the dictionary
  const int64_t dim = a.dim;
  const int tid = threadIdx.x;
  V* Rg = (V*)a.R;
  V* Pg = (V*)a.P;
  LancState* st = a.st;

  // --- Kronecker tables into LDS (after v)
  const H* aup = nullptr;
  const H* adw = nullptr;
  const H* upv = nullptr;
  const H* dwv = nullptr;
  const int32_t* upc = nullptr;
  const int32_t* dwc = nullptr;
  const uint8_t* impu = nullptr;
  const uint8_t* impd = nullptr;
  const double* uimp = nullptr;
  if constexpr (MODE == 1) {
    const KronArgs<HC>& K = a.K;
    unsigned char* q = smem + ((dim * sizeof(V) + 15) & ~(int64_t)15);
    auto carve = [&](int64_t bytes) {
      unsigned char* r = q;
      q += (bytes + 15) & ~(int64_t)15;
      return r;
    };
    H* s_aup = (H*)carve(K.dimup * sizeof(H));
    H* s_adw = (H*)carve(K.dimdw * sizeof(H));
    H* s_upv = (H*)carve((int64_t)K.degup * K.dimup * sizeof(H));
    H* s_dwv = (H*)carve((int64_t)K.degdw * K.dimdw * sizeof(H));
    int32_t* s_upc = (int32_t*)carve((int64_t)K.degup * K.dimup * 4);
    int32_t* s_dwc = (int32_t*)carve((int64_t)K.degdw * K.dimdw * 4);
    uint8_t* s_impu = (uint8_t*)carve(K.dimup);
    uint8_t* s_impd = (uint8_t*)carve(K.dimdw);
    double* s_uimp = (double*)carve((int64_t)K.nimp * K.nimp * 8);
    for (int64_t t = tid; t < K.dimup; t += NT) { s_aup[t] = K.aup[t]; s_impu[t] = K.impu[t]; }
    for (int64_t t = tid; t < K.dimdw; t += NT) { s_adw[t] = K.adw[t]; s_impd[t] = K.impd[t]; }
    for (int64_t t = tid; t < (int64_t)K.degup * K.dimup; t += NT) { s_upv[t] = K.upv[t]; s_upc[t] = K.upc[t]; }
    for (int64_t t = tid; t < (int64_t)K.degdw * K.dimdw; t += NT) { s_dwv[t] = K.dwv[t]; s_dwc[t] = K.dwc[t]; }
    for (int t = tid; t < K.nimp * K.nimp; t += NT) s_uimp[t] = K.uimp[t];
    aup = s_aup; adw = s_adw; upv = s_upv; dwv = s_dwv; upc = s_upc; dwc = s_dwc;
    impu = s_impu; impd = s_impd; uimp = s_uimp;
  }

  // --- MODE 2: dictionary | v | diagonal in LDS, ELL entries in registers.
  // (E is the row width W; the dictionary comes first so that its byte
  // offsets fit 14 bits; vl moves behind it)
  constexpr bool REG = MODE == 2 || MODE == 3;
  uint32_t pk[REG ? RPT * E : 1];
  // diagonal of a Hermitian H is real: kept as real(8) in LDS (host checks
  // the imaginary parts are zero before choosing a register mode)
  const double* dg = nullptr;
  const unsigned char* dct = smem;
  if constexpr (MODE == 2) {
    const int64_t dbytes = ((int64_t)a.ndict * sizeof(H) + 15) & ~(int64_t)15;
    for (int t = tid; t < a.ndict; t += NT) ((H*)smem)[t] = a.dict[t];
    vl = (V*)(smem + dbytes);
    double* s_g = (double*)(smem + dbytes + ((dim * sizeof(V) + 15) & ~(int64_t)15));
    for (int64_t t = tid; t < dim; t += NT) s_g[t] = re_of(a.diag[t]);
    dg = s_g;
#pragma unroll
    for (int k = 0; k < RPT * E; k++) pk[k] = a.pk[k * NT + tid];
  }
  if constexpr (MODE == 3) {
    // matrix-free: the ELL words are generated here from the Kronecker hop
    // tables (no matrix in HBM); the dictionary is the tables' value arrays
    // [upv | dwv | 0], so entry order and values are those of k_kron
    const KronArgs<HC>& K = a.K;
    const int du = (int)K.dimup, dd = (int)K.dimdw;
    const int nup = K.degup * du, ndw = K.degdw * dd;
    H* sd = (H*)smem;
    for (int t = tid; t < nup; t += NT) sd[t] = K.upv[t];
    for (int t = tid; t < ndw; t += NT) sd[nup + t] = K.dwv[t];
    if (tid == 0) sd[nup + ndw] = mk<HC>(0.0, 0.0);
    const int64_t dbytes = ((int64_t)(nup + ndw + 1) * sizeof(H) + 15) & ~(int64_t)15;
    vl = (V*)(smem + dbytes);
    double* s_g = (double*)(smem + dbytes + ((dim * sizeof(V) + 15) & ~(int64_t)15));
    for (int64_t t = tid; t < dim; t += NT) {
      const int iw = (int)(t / du), iu = (int)(t - (int64_t)iw * du);
      s_g[t] = re_of(add(add(K.aup[iu], K.adw[iw]), mk<HC>(K.uimp[K.impu[iu] * K.nimp + K.impd[iw]], 0.0)));
    }
    dg = s_g;
    const uint32_t hs = sizeof(H);
    const uint32_t zero = (uint32_t)((nup + ndw) * hs) << kPkColBits;
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int64_t i = tid + (int64_t)r * NT;
      const int iw = (int)(i / du), iu = (int)(i - (int64_t)iw * du);
#pragma unroll
      for (int e = 0; e < E; e++) {
        uint32_t wd = zero;
        if (i < dim) {
          if (e < K.degup) {
            const int q = e * du + iu;
            wd = (uint32_t)(iw * du + K.upc[q]) | (((uint32_t)q * hs) << kPkColBits);
          } else if (e < K.degup + K.degdw) {
            const int q = (e - K.degup) * dd + iw;
            wd = (uint32_t)(K.dwc[q] * du + iu) | (((uint32_t)(nup + q) * hs) << kPkColBits);
          }
        }
        pk[r * E + e] = wd;
      }
    }
  }

  // --- state in
  // complex vectors in register modes keep p = v_{k-1} in global memory (own
  // rows only, read once and written once per step, L2-resident): it frees
  // 4 VGPRs per row for the ELL words
  constexpr bool PG = REG && VC;
  V p[PG ? 1 : RPT];
  uint32_t rix[RPT];  // Kronecker row index packed (iw << 16) | iu  (DimUp, DimDw < 2^16)
  double b;
  int it0;
  {
    double nrm = 0.0;
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int64_t i = tid + (int64_t)r * NT;
      if constexpr (!PG) p[r] = vzero<V>();
      if (i < dim) {
        V x = Rg[i];
        vl[i] = x;
        if (a.first) {
          nrm += redot(x, x);
          if constexpr (PG) Pg[i] = vzero<V>();
        } else if constexpr (!PG) {
          p[r] = Pg[i];
        }
        if constexpr (MODE == 1) {
          const uint32_t w_ = (uint32_t)(i / a.K.dimup);
          rix[r] = (w_ << 16) | (uint32_t)(i - (int64_t)w_ * a.K.dimup);
        }
      }
    }
    if (a.first) {
      double n2 = pblock_sum<NT>(nrm, ws);  // includes barrier: vl complete
      if (n2 == 0.0) {                  // lanczos_plain_iteration: "norm =0!!"
        if (tid == 0) { st->iter = 0; st->done = 1; st->beta = 0.0; }
        return;
      }
      const double inv = 1.0 / sqrt(n2);
#pragma unroll
      for (int r = 0; r < RPT; r++) {
        const int64_t i = tid + (int64_t)r * NT;
        if (i < dim) vl[i] = scl(inv, vl[i]);
      }
      b = 0.0;
      it0 = 0;
      if (tid == 0) {
        st->iter = 0;
        st->done = 0;
        st->beta = 0.0;
      }
    } else {
      b = st->beta;
      it0 = st->iter;
    }
    __syncthreads();
  }
  if (st->done && !a.first) return;
  const double thresh = st->thresh;   // hoisted: a global read per iteration costs ~1 µs
  double* const alpha_out = a.alpha;
  double* const beta_out = a.beta;
  V* const basis = (V*)a.basis;

  for (int k = 0; k < a.niter; k++) {
    const int it = it0 + k;
    if constexpr (REG) {
      // entries are loop-invariant: keep the compiler from hoisting their
      // decoded addresses out of the iteration loop (2 VGPRs per entry)
#pragma unroll
      for (int e = 0; e < RPT * E; e++) asm volatile("" : "+v"(pk[e]));
    }
    // ---- w = H v - b p ; alpha partial
    V w[RPT];
    double ap = 0.0;
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int64_t i = tid + (int64_t)r * NT;
      w[r] = vzero<V>();
      if (i < dim) {
        const V xi = vl[i];
        V acc;
        if constexpr (MODE == 0) {
          const int64_t s = i >> 6, s0 = a.sptr[s];
          const int wd = (int)((a.sptr[s + 1] - s0) >> 6);
          const int32_t* cp = a.cols + s0 + (i & 63);
          const H* vp = a.vals + s0 + (i & 63);
          acc = add(vzero<V>(), mul(a.diag[i], xi));
          for (int k0 = 0; k0 < wd; k0 += kPChunk) {
            int32_t c[kPChunk];
            H h[kPChunk];
#pragma unroll
            for (int kk = 0; kk < kPChunk; kk++) c[kk] = (k0 + kk < wd) ? cp[64 * (k0 + kk)] : 0;
#pragma unroll
            for (int kk = 0; kk < kPChunk; kk++)
              h[kk] = (k0 + kk < wd) ? vp[64 * (k0 + kk)] : mk<HC>(0.0, 0.0);
#pragma unroll
            for (int kk = 0; kk < kPChunk; kk++)
              if (k0 + kk < wd) acc = add(acc, mul(h[kk], vl[c[kk]]));
          }
        } else if constexpr (REG) {
          acc = mul(dg[i], xi);
#pragma unroll
          for (int e = 0; e < E; e++) {
            const uint32_t x = pk[r * E + e];
            const H h = *(const H*)(dct + ((x >> kPkColBits) & kPkOffMask));
            acc = fmac(acc, h, vl[x & kPkColMask]);
          }
        } else {
          const int du = (int)a.K.dimup, dd = (int)a.K.dimdw;
          const int iwr = (int)(rix[r] >> 16), iur = (int)(rix[r] & 0xffffu);
          auto d = add(add(aup[iur], adw[iwr]), mk<HC>(uimp[impu[iur] * a.K.nimp + impd[iwr]], 0.0));
          acc = mul(d, xi);
          const V* xrow = vl + iwr * du;
          for (int kk = 0; kk < a.K.degup; kk++) {
            const int q = kk * du + iur;
            acc = add(acc, mul(upv[q], xrow[upc[q]]));
          }
          for (int kk = 0; kk < a.K.degdw; kk++) {
            const int q = kk * dd + iwr;
            acc = add(acc, mul(dwv[q], vl[dwc[q] * du + iur]));
          }
        }
        if constexpr (PG) w[r] = sub(acc, scl(b, Pg[i]));
        else w[r] = sub(acc, scl(b, p[r]));
        ap += redot(xi, w[r]);
        if (basis) basis[(int64_t)it * dim + i] = xi;
      }
    }
    // alpha reads ws, beta ws2; the barrier inside the beta reduction and the
    // end-of-step barrier separate each read from the next write of its buffer
    const double alpha = pblock_sum<NT, false>(ap, ws);
    // ---- w -= alpha v ; beta
    double bp = 0.0;
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int64_t i = tid + (int64_t)r * NT;
      if (i < dim) {
        w[r] = sub(w[r], scl(alpha, vl[i]));
        bp += redot(w[r], w[r]);
      }
    }
    const double bn = sqrt(pblock_sum<NT, false>(bp, ws2));
    if (tid == 0) {
      alpha_out[it] = alpha;
      beta_out[it + 1] = bn;
    }
    const bool stop = bn < thresh;
    // ---- p <- v ; v <- w / b
    const double inv = 1.0 / bn;
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int64_t i = tid + (int64_t)r * NT;
      if (i < dim) {
        if constexpr (PG) Pg[i] = vl[i];
        else p[r] = vl[i];
        vl[i] = scl(inv, w[r]);
      }
    }
    b = bn;
    __syncthreads();
    if (stop) {
      if (tid == 0) {
        st->done = 1;
        st->iter = it + 1;
        st->beta = bn;
      }
      return;
    }
  }
  // ---- state out
#pragma unroll
  for (int r = 0; r < RPT; r++) {
    const int64_t i = tid + (int64_t)r * NT;
    if (i < dim) {
      Rg[i] = vl[i];
      if constexpr (!PG) Pg[i] = p[r];
    }
  }
  if (tid == 0) {
    st->iter = it0 + a.niter;
    st->beta = b;
  }
}

}  // namespace edg
