// ed_persist.hpp — one-workgroup persistent Lanczos for small sectors.
//
// For sectors whose Lanczos vector fits in LDS (configs[1]: dim 4,900 real =
// 39 KB) the per-iteration cost of the multi-kernel recurrence is launch and
// grid-reduction latency, not bandwidth (≈9 µs per iteration for 4,900 rows).
// Here one workgroup (one CU) runs many iterations of the
// .repo/PLAIN_LANCZOS.f90:87-118 recurrence without leaving the CU:
//   * r_k = b_k v_k (unnormalised) lives in LDS and is gathered by the H·v;
//     p = v_{k-1}, w and (real vectors) the own rows of r_k live in registers
//     of the thread that owns the row; every thread owns RPT row slots, padded
//     to NT*RPT rows with zero entries so that no per-row branch exists;
//   * H is the stored SELL-64 matrix streamed from L2 (MODE 0), the Kronecker
//     tables copied into LDS (MODE 1, normal mode without Jx/Jp), the stored
//     matrix held in REGISTERS as ELL words {col:17 | value byte offset:14}
//     into an LDS dictionary of the distinct values (MODE 2), the same words
//     generated in-kernel from the Kronecker hop tables (MODE 3), or the
//     Kronecker register layout (MODE 4, real H and vectors): thread (g, iu)
//     owns rows (iw = g + G*r, iu), keeps its up-hop list (target, value) once
//     and per row the down-hop entries and the diagonal — no dictionary, the
//     down-hop gathers of a wavefront are contiguous;
//   * alpha and beta are block reductions (DPP wave sums + one LDS stage),
//     two barriers per iteration, no global synchronisation.
// configs[1]: MODE 4 1.87 µs per step with the slot-major LDS vector below
// (2.24 before it; MODE 2 4.4 µs before the Kronecker layout).
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
  // Kronecker tables (MODE 1, 3; MODE 4 direct diagonal)
  KronArgs<HC> K;
  int64_t dim;
  void* R;           // in: start vector (first) or saved unnormalised r_k; out: saved r_k
  void* P;           // saved p = v_{k-1}
  LancState* st;     // beta (norm of R), iter, done
  double* alpha;     // [niter_total]
  double* beta;      // [niter_total+1]
  void* basis;       // optional Krylov basis (column k = v_k), or null
  // register-resident stored matrix (MODE 2)
  const uint32_t* pk;   // [RPT*W][kPRegBlock] packed entries
  const H* dict;        // [ndict] distinct values, dict[0] = 0
  int ndict;
  // Kronecker register layout (MODE 4): per-spin hop lists [deg][n] (target
  // rank, value), zero-padded beyond a row's own degree
  const int32_t* kupc;
  const double* kupv;
  const int32_t* kdwc;
  const double* kdwv;
  const double* kdiag;  // [dim] real diagonal, or null: from K (aup + adw + U)
  int kdu, kdd, kdegu, kdegd;
  double thresh;     // breakdown threshold (|b| < thresh stops)
  int niter;         // iterations in this launch
  int first;         // 1: R holds the unnormalised start vector
  // batched launches (one workgroup per run, same H): run b = blockIdx.x uses
  // R + b*ldr, P + b*ldp, st + b, alpha/beta + b*ldab (0: single run)
  int64_t ldr, ldp;
  int64_t ldab;
};

// Wave sum on DPP row operations (no LDS traffic, ~6 dependent VALU steps
// instead of 6 ds_bpermute round trips); the total lands in lane 63.
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_add(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int l2 = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, 0xF, false);
  const int h2 = __builtin_amdgcn_update_dpp(0, hi, CTRL, RM, 0xF, false);
  return v + __hiloint2double(h2, l2);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v = dpp_add<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v = dpp_add<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v = dpp_add<0x141, 0xF>(v);  // row_half_mirror
  v = dpp_add<0x140, 0xF>(v);  // row_mirror: every lane holds its row's sum
  v = dpp_add<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v = dpp_add<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  return v;
}

// Deterministic block sum (fixed order), valid in every thread.  Must be
// reached by all threads with full waves (DPP).  TAIL=false drops the
// trailing barrier: the caller guarantees a barrier between this read of ws
// and the next write to the same buffer.
template <int NT = kPBlock, bool TAIL = true>
__device__ __forceinline__ double pblock_sum(double v, double* ws) {
  v = wave_sum_dpp(v);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) t = t + ws[w];
  if constexpr (TAIL) __syncthreads();
  return t;
}

constexpr uint32_t kPkColBits = 17, kPkColMask = (1u << kPkColBits) - 1;
constexpr uint32_t kPkOffMask = (1u << 14) - 1;  // dictionary byte offset (<= 16 KiB)

// Absolute LDS addressing for MODE 4's gathers: the byte address of an LDS
// object, and loads through such an address — a constant added to it folds
// into the ds_read immediate offset (no per-gather address add) when the
// compiler can see the address is non-negative (masked at setup).
__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
template <typename T>
__device__ __forceinline__ T lds_ldv(uint32_t a) {
  if constexpr (sizeof(T) == 16) {
    // through the native 2-vector type: one ds_read_b128 (a HIP_vector_type
    // load is split into two 8-B loads, a ds_read2_b64 at twice the cycles)
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v v = *(const __attribute__((address_space(3))) d2v*)(uintptr_t)a;
    return T{v.x, v.y};
  } else {
    return *(const __attribute__((address_space(3))) T*)(uintptr_t)a;
  }
}

// Rows of one thread: slot r holds row row0 + r*stride; slots r < nvalid are
// basis rows (< dim), the others are padding rows in [dim, NT*RPT) whose LDS
// entries, diagonal and matrix entries are zero, so every loop over r runs
// without a branch (no per-row EXEC save / LDS wait).
struct PRows {
  int row0, stride, nvalid, iu;
};

template <int MODE, int RPT, int NT>
__device__ __forceinline__ PRows persist_rows(int tid, int64_t dim, int du, int dd) {
  PRows q;
  if constexpr (MODE == 4) {
    // Kronecker layout: thread (g, iu) owns rows (iw = g + G*r, iu), so its
    // up-hop list is the same for all of its rows
    const int G = NT / du;
    if (tid < G * du) {
      const int g = tid / du;
      q.iu = tid - g * du;
      q.row0 = g * du + q.iu;
      q.stride = G * du;
      q.nvalid = dd > g ? (dd - g + G - 1) / G : 0;
    } else {  // idle lanes: private padding rows above G*du*RPT
      q.iu = 0;
      q.row0 = G * du * RPT + (tid - G * du);
      q.stride = NT - G * du;
      q.nvalid = 0;
    }
  } else {
    q.iu = 0;
    q.row0 = tid;
    q.stride = NT;
    q.nvalid = dim > tid ? (int)((dim - tid + NT - 1) / NT) : 0;
  }
  return q;
}

// One-workgroup plain Lanczos (.repo/PLAIN_LANCZOS.f90:87-118):
//   w = H v_k - b_k v_{k-1};  a_k = <v_k, w>;  w -= a_k v_k;  b_{k+1} = |w|
// LDS holds r_k = b_k v_k UNNORMALISED: w is stored as soon as a_k is known
// (all gathers of the step are behind the alpha barrier) and the next step
// scales H r by 1/b — two barriers per step (alpha, beta), one LDS vector.
template <bool HC, bool VC, int MODE, int RPT, int E = 1, int NT = kPBlock>
__global__ void __launch_bounds__(NT) k_lanc_persist(const PersistRun<HC> a) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ double ws[NT / 64];
  __shared__ double ws2[NT / 64];
  constexpr int VROWS = NT * RPT;  // LDS vector rows incl. padding
  // MODE 4: slot-major LDS vector — row slot r of thread t at element
  // r * VSLOT + t, VSLOT = NT + 1 (consecutive slots are 8 B off a 512-B
  // multiple, so two slots' reads never merge into one ds_read2st64, which
  // costs what two ds_read_b64 do twice over); a gather of slot r then
  // addresses through a per-lane base plus the immediate r * VSLOT * size.
  // (Not the complex-vector form: measured ~3 % slower per step (3.94-3.98
  // against 3.82-3.86 us) and 18 % slower batched with it; that form keeps
  // the natural row order.)
  constexpr bool SLOT = MODE == 4 && !VC;
  constexpr int VSLOT = NT + 1;
  constexpr int VLDS = SLOT ? RPT * VSLOT : VROWS;  // LDS vector elements
  V* vl = (V*)smem;                // MODE 2/3 move it behind the dictionary
  const int64_t dim = a.dim;
  const int tid = threadIdx.x;
  const int run = blockIdx.x;  // batched launches: one independent run per workgroup
  V* Rg = (V*)a.R + run * a.ldr;
  V* Pg = (V*)a.P + run * a.ldp;
  LancState* st = a.st + run;
  PRows q = persist_rows<MODE, RPT, NT>(tid, dim, a.kdu, a.kdd);
#define PROW(r) (q.row0 + (r) * q.stride)
#define LPOS(r) (SLOT ? (r) * VSLOT + tid : PROW(r))

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
    unsigned char* qq = smem + (((int64_t)VROWS * sizeof(V) + 15) & ~(int64_t)15);
    auto carve = [&](int64_t bytes) {
      unsigned char* r = qq;
      qq += (bytes + 15) & ~(int64_t)15;
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

  // --- MODE 2/3: dictionary | v | diagonal in LDS, ELL entries in registers.
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
    double* s_g = (double*)(smem + dbytes + (((int64_t)VROWS * sizeof(V) + 15) & ~(int64_t)15));
    for (int t = tid; t < VROWS; t += NT) s_g[t] = t < dim ? re_of(a.diag[t]) : 0.0;
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
    double* s_g = (double*)(smem + dbytes + (((int64_t)VROWS * sizeof(V) + 15) & ~(int64_t)15));
    for (int t = tid; t < VROWS; t += NT) {
      const int iw = t / du, iu = t - iw * du;
      s_g[t] = t < dim ? re_of(add(add(K.aup[iu], K.adw[iw]), mk<HC>(K.uimp[K.impu[iu] * K.nimp + K.impd[iw]], 0.0)))
                       : 0.0;
    }
    dg = s_g;
    const uint32_t hs = sizeof(H);
    const uint32_t zero = (uint32_t)((nup + ndw) * hs) << kPkColBits;
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int i = PROW(r);
      const int iw = i / du, iu = i - iw * du;
#pragma unroll
      for (int e = 0; e < E; e++) {
        uint32_t wd = zero;
        if (r < q.nvalid) {
          if (e < K.degup) {
            const int qq = e * du + iu;
            wd = (uint32_t)(iw * du + K.upc[qq]) | (((uint32_t)qq * hs) << kPkColBits);
          } else if (e < K.degup + K.degdw) {
            const int qq = (e - K.degup) * dd + iw;
            wd = (uint32_t)(K.dwc[qq] * du + iu) | (((uint32_t)(nup + qq) * hs) << kPkColBits);
          }
        }
        pk[r * E + e] = wd;
      }
    }
  }
  if constexpr (REG) {
    // words -> absolute LDS addresses {v entry: 17 bits | dictionary entry:
    // 15 bits} (v ends below 128 KiB and the dictionary below 32 KiB in every
    // layout the host admits): the loop then takes each address with one
    // AND or one shift instead of a mask, a shift-add and a base add apiece
    const uint32_t lbv = lds_addr_of(vl), lbd = lds_addr_of(dct);
#pragma unroll
    for (int k = 0; k < RPT * E; k++) {
      const uint32_t x = pk[k];
      pk[k] = (lbv + (x & kPkColMask) * (uint32_t)sizeof(V)) |
              ((lbd + ((x >> kPkColBits) & kPkOffMask)) << kPkColBits);
    }
  }
  // --- MODE 4: Kronecker register layout (real H).  Up-hop list (target
  // rank as a byte offset inside the V row, value) once per thread; down-hop
  // entries (LDS byte address, value) and the diagonal per row; no
  // dictionary, no matrix byte in LDS.  Complex vectors (the reference's
  // complex(8) arithmetic on a real H; KRC): the up-hop values and the
  // diagonal in registers as for real vectors, the down-hop values read from
  // a [slot][iw] table behind the vector in LDS (lanes of one iw broadcast)
  // instead of registers, whose budget the complex w take; p = v_{k-1} in
  // global memory.  (Round 3's 1,024-thread complex layout, 4.10 us per
  // configs[1] step against 3.83-3.86, was removed in round 5.)
  constexpr bool KR = MODE == 4;
  constexpr bool KRC = KR && VC;
  uint32_t ucol[KR ? E : 1];  // KR: absolute LDS byte address of the up-hop target in slot 0
  double uval[KR ? E : 1];
  uint32_t dcol[KR ? RPT * E : 1];  // KR: absolute LDS byte address of the down-hop target
  double dval[(KR && !VC) ? RPT * E : 1];
  double dgr[KR ? RPT : 1];
  const double* sdv = nullptr;   // KRC: down-hop values [e * dd + iw]
  int giw = 0;                   // KR: g of the thread (row slot r has iw = g + G*r)
  if constexpr (KR) {
    const int du = a.kdu, dd = a.kdd, G = NT / du;
    const bool act = tid < G * du;
    const int g = act ? tid / du : 0;
    giw = g;
    if constexpr (KRC) {
      // LDS: vector | down-hop values [e * dd + iw]
      double* t = (double*)(smem + (((int64_t)VLDS * sizeof(V) + 15) & ~(int64_t)15));
      for (int x = tid; x < E * dd; x += NT) t[x] = x < a.kdegd * dd ? a.kdwv[x] : 0.0;
      sdv = t;
    }
    const uint32_t lb = lds_addr_of(vl);
    constexpr uint32_t kLdsMask = (1u << 18) - 1;  // LDS byte addresses < 256 KiB: known non-negative
#pragma unroll
    for (int e = 0; e < E; e++) {
      const bool ok = act && e < a.kdegu;
      // idle lanes read their own (zero) padding slot; padded hops a real
      // entry of the row times a zero value
      if constexpr (SLOT) {
        const int pos = act ? g * du + (ok ? a.kupc[e * du + q.iu] : 0) : tid;
        // (the mask also states the element alignment: b128 loads stay whole)
        ucol[e] = (lb + (uint32_t)pos * (uint32_t)sizeof(V)) & kLdsMask & ~(uint32_t)(sizeof(V) - 1);
      } else {  // byte offset inside the row iw (the row base added per row slot)
        ucol[e] = ok ? (uint32_t)a.kupc[e * du + q.iu] * (uint32_t)sizeof(V) : 0u;
      }
      uval[e] = ok ? a.kupv[e * du + q.iu] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const bool okr = r < q.nvalid;
      const int iw = g + G * r;
#pragma unroll
      for (int e = 0; e < E; e++) {
        const bool ok = okr && e < a.kdegd;
        // target row (iw', iu) sits in slot iw' / G of thread (iw' % G, iu)
        int pos;
        if (ok) {
          const int iw2 = a.kdwc[e * dd + iw], r2 = iw2 / G;
          pos = SLOT ? r2 * VSLOT + (iw2 - r2 * G) * du + q.iu : iw2 * du + q.iu;
        } else {
          // padding slots gather their own (zero) slot, valid rows beyond
          // their degree element 0 times a zero value
          pos = okr ? 0 : LPOS(r);
        }
        // (natural layout: a byte offset from vl, as before the slot layout)
        dcol[r * E + e] = (SLOT ? lb : 0u) + (uint32_t)pos * (uint32_t)sizeof(V);
        if constexpr (!(KR && VC)) dval[r * E + e] = ok ? a.kdwv[e * dd + iw] : 0.0;
      }
      {
        double d = 0.0;
        if (okr) {
          if (a.kdiag) {
            d = a.kdiag[PROW(r)];
          } else {
            const KronArgs<HC>& K = a.K;
            d = re_of(add(add(K.aup[q.iu], K.adw[iw]), mk<HC>(K.uimp[K.impu[q.iu] * K.nimp + K.impd[iw]], 0.0)));
          }
        }
        dgr[r] = d;
      }
    }
  }

  // --- state in
  // complex vectors in register modes keep p = v_{k-1} in global memory (own
  // rows only, read once and written once per step, L2-resident): it frees
  // 4 VGPRs per row for the ELL words.  P is allocated with >= NT*RPT rows
  // (p_rows, ed_lib.hip) so padding slots load and store without a guard.
  constexpr bool PG = (REG || KRC) && VC;
  // real vectors keep their own rows of r_k in registers; complex ones
  // re-read them from LDS (register budget of the ELL words)
  // (MODE 4 at 10 rows per thread reads them from LDS with the gathers: the
  // software-pipelined gathers need the 20 VGPRs)
  constexpr bool PIPE = KR && !VC && RPT * E <= 40;  // software-pipelined MODE 4 gathers (spill-free)
  constexpr bool UREG = !VC && (REG || (KR && (!PIPE || RPT * E < 40)));
  V u[UREG ? RPT : 1];  // own rows of r_k (the LDS vector)
  V p[PG ? 1 : RPT];
  uint32_t rix[RPT];    // Kronecker row index packed (iw << 16) | iu  (DimUp, DimDw < 2^16)
  double b, s;          // b_k and 1/b_k (s = 1/|r_0| on the first step, b_0 = 0)
  int it0;
  {
    double nrm = 0.0;
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int i = PROW(r);
      const bool ok = r < q.nvalid;
      const V x = ok ? Rg[i] : vzero<V>();
      if constexpr (UREG) u[r] = x;
      vl[LPOS(r)] = x;
      if constexpr (!PG) p[r] = (ok && !a.first) ? Pg[i] : vzero<V>();
      if (a.first) {
        nrm += redot(x, x);
        if constexpr (PG) Pg[i] = vzero<V>();  // padding rows too
      }
      if constexpr (MODE == 1) {
        const uint32_t w_ = (uint32_t)(i / a.K.dimup);
        rix[r] = ok ? (w_ << 16) | (uint32_t)(i - (int64_t)w_ * a.K.dimup) : 0u;
      }
    }
    if (a.first) {
      const double n2 = pblock_sum<NT>(nrm, ws);
      if (n2 == 0.0) {                  // lanczos_plain_iteration: "norm =0!!"
        if (tid == 0) { st->iter = 0; st->done = 1; st->beta = 0.0; }
        return;
      }
      s = 1.0 / sqrt(n2);
      b = 0.0;
      it0 = 0;
      if (tid == 0) {
        st->iter = 0;
        st->done = 0;
        st->beta = 0.0;
      }
    } else {
      b = st->beta;
      s = 1.0 / b;
      it0 = st->iter;
    }
    __syncthreads();
  }
  if (st->done && !a.first) return;
  const double thresh = a.thresh;
  double* const alpha_out = a.alpha + run * a.ldab;
  double* const beta_out = a.beta + run * a.ldab;
  V* const basis = run == 0 ? (V*)a.basis : nullptr;

  for (int k = 0; k < a.niter; k++) {
    const int it = it0 + k;
    if constexpr (REG) {
      // entries are loop-invariant: keep the compiler from hoisting their
      // decoded addresses out of the iteration loop (2 VGPRs per entry)
#pragma unroll
      for (int e = 0; e < RPT * E; e++) asm volatile("" : "+v"(pk[e]));
    }
    if constexpr (KR) {
#pragma unroll
      for (int e = 0; e < RPT * E; e++) asm volatile("" : "+v"(dcol[e]));
    }
    // opaque row base: the per-row LDS / global addresses are re-derived each
    // step (one integer op) instead of being hoisted into 1-2 VGPRs per row
    asm volatile("" : "+v"(q.row0));
    // ---- w = (H r_k)/b_k - b_k p ; alpha partial
    V w[RPT];
    double ap = 0.0;
    if constexpr (PIPE) {
      // MODE 4: software-pipelined gathers — row r+1's 2E LDS reads are in
      // flight while row r is summed (issued per hop group of 4 and waited
      // at once, one wave had <= 4 reads outstanding: the LDS latency was
      // exposed ~20 times per step at 2 waves per SIMD)
      double gu[E], gd[E], go;
      auto gather = [&](int r, double* hu, double* hd, double& ho) {
#pragma unroll
        for (int e = 0; e < E; e++) hu[e] = lds_ldv<double>(ucol[e] + r * VSLOT * 8);  // slot r of row iw
#pragma unroll
        for (int e = 0; e < E; e++) hd[e] = lds_ldv<double>(dcol[r * E + e]);
        if constexpr (UREG) ho = u[r];
        else ho = vl[LPOS(r)];
      };
      gather(0, gu, gd, go);
#pragma unroll
      for (int r = 0; r < RPT; r++) {
        double nu[E], nd[E], no = 0.0;
        if (r + 1 < RPT) gather(r + 1, nu, nd, no);
        const double ur = go;
        double acc = ur * dgr[r];
#ifndef ED_P4_NOGATHER  // timing probe: the step without its gathers
#pragma unroll
        for (int e = 0; e < E; e++) acc = fma(uval[e], gu[e], acc);
#pragma unroll
        for (int e = 0; e < E; e++) acc = fma(dval[r * E + e], gd[e], acc);
#endif
        // contracted recurrence (MODE 4 already fuses its gathers; the
        // Lanczos bar is 1e-10, not bit-exactness): f64 VALU issue is a
        // large part of the step at 2 waves per SIMD
        const double x = s * ur;
        w[r] = fma(s, acc, -(b * p[r]));
        ap = fma(x, w[r], ap);
        if (r + 1 < RPT) {
#pragma unroll
          for (int e = 0; e < E; e++) {
            gu[e] = nu[e];
            gd[e] = nd[e];
          }
          go = no;
        }
      }
    } else {
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int i = PROW(r);
      const V ur = UREG ? u[r] : vl[LPOS(r)];
      V acc;
      if constexpr (MODE == 0) {
        acc = vzero<V>();
        if (r < q.nvalid) {
          const int64_t sl = i >> 6, s0 = a.sptr[sl];
          const int wd = (int)((a.sptr[sl + 1] - s0) >> 6);
          const int32_t* cp = a.cols + s0 + (i & 63);
          const H* vp = a.vals + s0 + (i & 63);
          acc = add(vzero<V>(), mul(a.diag[i], ur));
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
        }
      } else if constexpr (REG) {
        acc = mul(dg[i], ur);
#pragma unroll
        for (int e = 0; e < E; e++) {
          const uint32_t x = pk[r * E + e];
          const H h = lds_ldv<H>(x >> kPkColBits);
          acc = fmac(acc, h, lds_ldv<V>(x & kPkColMask));
        }
      } else if constexpr (KR) {
        acc = mul(dgr[r], ur);
        {
        if constexpr (SLOT) {
#pragma unroll
          for (int e = 0; e < E; e++) acc = fmac(acc, uval[e], lds_ldv<V>(ucol[e] + r * VSLOT * (int)sizeof(V)));
        } else {
          const unsigned char* rb = (const unsigned char*)(vl + (i - q.iu));  // row iw of V
#pragma unroll
          for (int e = 0; e < E; e++) acc = fmac(acc, uval[e], *(const V*)(rb + ucol[e]));
        }
        if constexpr (KR && VC) {
          const int iwc = min(giw + (NT / a.kdu) * r, a.kdd - 1);
#pragma unroll
          for (int e = 0; e < E; e++)
            acc = fmac(acc, sdv[e * a.kdd + iwc],
                       SLOT ? lds_ldv<V>(dcol[r * E + e]) : *(const V*)((const unsigned char*)vl + dcol[r * E + e]));
        } else {
#pragma unroll
          for (int e = 0; e < E; e++)
            acc = fmac(acc, dval[r * E + e], lds_ldv<V>(dcol[r * E + e]));
        }
        }
      } else {
        acc = vzero<V>();
        if (r < q.nvalid) {
          const int du = (int)a.K.dimup, dd = (int)a.K.dimdw;
          const int iwr = (int)(rix[r] >> 16), iur = (int)(rix[r] & 0xffffu);
          auto d = add(add(aup[iur], adw[iwr]), mk<HC>(uimp[impu[iur] * a.K.nimp + impd[iwr]], 0.0));
          acc = mul(d, ur);
          const V* xrow = vl + iwr * du;
          for (int kk = 0; kk < a.K.degup; kk++) {
            const int qq = kk * du + iur;
            acc = add(acc, mul(upv[qq], xrow[upc[qq]]));
          }
          for (int kk = 0; kk < a.K.degdw; kk++) {
            const int qq = kk * dd + iwr;
            acc = add(acc, mul(dwv[qq], vl[dwc[qq] * du + iur]));
          }
        }
      }
      const V x = scl(s, ur);  // v_k
      V pr;
      if constexpr (PG) pr = Pg[i];  // P has >= NT*RPT rows, padding zero
      else pr = p[r];
      w[r] = sub(scl(s, acc), scl(b, pr));
      ap += redot(x, w[r]);
    }
    }
    // alpha barrier: every gather of r_k in LDS is done -> r_k's slots may
    // be overwritten by w below
#ifdef ED_P4_NOALPHA  // timing probe: the step without the alpha reduction (a bare barrier)
    __syncthreads();
    const double alpha = ap * 1e-300;
#else
    const double alpha = pblock_sum<NT, false>(ap, ws);
#endif
    // ---- w -= alpha v ; beta ; p <- v_k ; publish w (= r_{k+1}) in LDS
    double bp = 0.0;
    if (basis) {  // uniform: no per-row EXEC masking when no basis is kept
#pragma unroll
      for (int r = 0; r < RPT; r++)
        if (r < q.nvalid) basis[(int64_t)it * dim + PROW(r)] = scl(s, UREG ? u[r] : vl[LPOS(r)]);  // column k = v_k
    }
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int i = PROW(r);
      const V x = scl(s, UREG ? u[r] : vl[LPOS(r)]);
      if constexpr (PIPE) {
        w[r] = fma(-alpha, x, w[r]);
        bp = fma(w[r], w[r], bp);
      } else {
        w[r] = sub(w[r], scl(alpha, x));
        bp += redot(w[r], w[r]);
      }
      if constexpr (PG) {
        Pg[i] = x;
      } else {
        p[r] = x;
      }
      if constexpr (UREG) u[r] = w[r];
      vl[LPOS(r)] = w[r];
    }
    // beta barrier: also publishes r_{k+1}
#ifdef ED_P4_NOBETA  // timing probe: the step without the beta reduction (a bare barrier)
    __syncthreads();
    const double bn = 1.0 + bp * 1e-300;
#else
    const double bn = sqrt(pblock_sum<NT, false>(bp, ws2));
#endif
    if (tid == 0) {
      alpha_out[it] = alpha;
      beta_out[it + 1] = bn;
    }
    b = bn;
    s = 1.0 / bn;
    if (bn < thresh) {
      if (tid == 0) {
        st->done = 1;
        st->iter = it + 1;
        st->beta = bn;
      }
      return;
    }
  }
  // ---- state out: R = r_k (unnormalised), P = v_{k-1}, st->beta = b_k
#pragma unroll
  for (int r = 0; r < RPT; r++) {
    if (r < q.nvalid) {
      Rg[PROW(r)] = UREG ? u[r] : vl[LPOS(r)];
      if constexpr (!PG) Pg[PROW(r)] = p[r];
    }
  }
  if (tid == 0) {
    st->iter = it0 + a.niter;
    st->beta = b;
  }
#undef PROW
#undef LPOS
}

}  // namespace edg
