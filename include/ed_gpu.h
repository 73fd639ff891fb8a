/*
 * ed_gpu.h — C-ABI of the MI355X-native Lanczos H·v hot path for dmft-ed.
 *
 * This is the drop-in boundary.  Every entry point is `extern "C"`, takes plain
 * pointers and sizes, returns an int status (ED_OK = 0) and leaves a message in
 * ed_gpu_last_error() on failure.  Nothing here mentions torch or HIP types:
 * streams are passed as `void*` (a hipStream_t, or NULL for the default stream).
 *
 * Two layers:
 *   1. Reference-shaped global API (ed_gpu_init / ed_gpu_build_sector /
 *      ed_gpu_hxv / ed_gpu_delete_sector ...).  It keeps one "current sector",
 *      exactly like the module state Hsector/H/spH0 of the reference, so that a
 *      Fortran procedure pointer with the cc_sparse_HxV interface can call it
 *      unchanged (see dmft-ed_amd/fortran/ed_gpu_hxv.f90 and INTEGRATION.md).
 *   2. Handle API (ed_sector_*) used by the sector / Green's-function seed farm,
 *      where many sectors live at once on several GPUs.
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   ed_params                 <- effective_bath (ED_VARS_GLOBAL.f90:12-22), impHloc
 *                                (ED_VARS_GLOBAL.f90:73), Uloc/Ust/Jh/Jx/Jp/xmu/hfmode
 *                                (ED_INPUT_VARS.f90:17-31), Jhflag (ED_SETUP.f90:289-290)
 *   ed_gpu_build_sector       <- build_Hv_sector        ED_HAMILTONIAN.f90:42-103
 *                                (+ build_sector ED_SETUP.f90:886-984,
 *                                   ed_buildH_c ED_HAMILTONIAN_STORED_HxV.f90:28-113)
 *   ed_gpu_hxv                <- cc_sparse_HxV          ED_VARS_GLOBAL.f90:48-54
 *                                = spMatVec_cc          ED_HAMILTONIAN_STORED_HxV.f90:132-143
 *                                / directMatVec_cc      ED_HAMILTONIAN_DIRECT_HxV.f90:21-92
 *   ed_gpu_delete_sector      <- delete_Hv_sector       ED_HAMILTONIAN.f90:106-123
 *                                (safe after a direct build, unlike the reference)
 *   ed_gpu_vecdim             <- vecDim_Hv_sector       ED_HAMILTONIAN.f90:126-149
 *   ed_gpu_dump_csr           <- sp_dump_matrix         ED_SPARSE_MATRIX.f90:331-388
 *                                (row-of-arrays order of sp_insert_element :249-320)
 *   ed_gpu_lanc_eigh          <- sp_lanc_eigh (SciFortran; spec .repo/PLAIN_LANCZOS.f90:286-385)
 *   ed_gpu_lanc_tridiag       <- sp_lanc_tridiag (SciFortran; spec .repo/PLAIN_LANCZOS.f90:154-180)
 *   ed_gpu_eigh               <- sp_eigh (ARPACK; called at ED_DIAG.f90:145-167)
 */
#ifndef ED_GPU_H
#define ED_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- limits */
#define ED_MAX_NORB  3   /* ed_checks_global: Norb<=3  (ED_SETUP.f90:56) */
#define ED_MAX_NSPIN 2   /* ed_checks_global: Nspin<=2 (ED_SETUP.f90:55) */
#define ED_MAX_NBATH 32
#define ED_MAX_NS    16  /* levels per spin: states are 2*Ns <= 32 bit words */

/* ---------------------------------------------------------------- enums */
#define ED_MODE_NORMAL 0 /* ed_mode='normal' : sectors (nup,ndw)        */
#define ED_MODE_SUPERC 1 /* ed_mode='superc' : sectors sz = nup-ndw     */
#define ED_MODE_NONSU2 2 /* ed_mode='nonsu2' : sectors n  = nup+ndw     */

#define ED_BATH_NORMAL  0 /* bath_type='normal'  */
#define ED_BATH_HYBRID  1 /* bath_type='hybrid'  */
#define ED_BATH_REPLICA 2 /* bath_type='replica' */

/* build flags (bit set) */
#define ED_STORED 0x1 /* ed_sparse_H=T: assemble H on the device (SELL-64 layout) */
#define ED_DIRECT 0x2 /* ed_sparse_H=F: matrix-free H·v, elements regenerated     */
#define ED_REAL   0x4 /* store H as real(8) (only when impHloc and bath are real) */
#define ED_NO_PACK   0x10 /* stored: plain SELL arrays only (no {col|value index} words) */
#define ED_KRON2_OFF 0x20 /* matrix-free Kronecker form: one-pass k_kron only       */
#define ED_KRON2_ON  0x40 /* two-pass Kronecker tables below the size threshold too */
#define ED_NO_SPLIT  0x80 /* stored: no two-segment form (one-pass k_spmv_pk only)          */
#define ED_SPLIT_ON  0x100 /* stored: two-segment form below the size threshold too        */
#define ED_FUSED_ON  0x200 /* stored: fused one-pass re-laid form below the size threshold too */
#define ED_NO_FUSED  0x400 /* stored: no fused one-pass re-laid form                       */

/* Kernel-selection options of a built sector (ed_sector_set_options): the
 * alternatives kept for parity tests and A/B measurements.  0 = the default
 * choice everywhere; nothing in the library reads the environment.  Bits
 * 0x010, 0x400, 0x8000 and 0x10000-0x80000 belonged to alternatives measured
 * slower and removed in round 5 (DESIGN.md keeps their numbers); they are
 * rejected as unknown. */
#define ED_OPT_NO_PERSIST     0x001 /* Lanczos: graph-captured multi-kernel recurrence only   */
#define ED_OPT_PERSIST_STORED 0x002 /* Lanczos: persistent MODE 0 (stored matrix from L2)      */
#define ED_OPT_NO_PREG        0x004 /* Lanczos: no register-resident modes (2, 3, 4)           */
#define ED_OPT_NO_PKRON       0x008 /* Lanczos: no Kronecker register layout (MODE 4)          */
#define ED_OPT_SPLIT_SIMPLE   0x020 /* kron_rows/cols: one-thread-per-row kernels              */
#define ED_OPT_NO_BATCH       0x040 /* lanc_tridiag_batch: seeds one after the other           */
#define ED_OPT_EIGH_NO_VERIFY 0x080 /* eigh: no deflated search for missed degenerate copies   */
#define ED_OPT_TRLAN_UNFUSED  0x100 /* eigh: four-sweep CGS2 instead of the fused sweeps       */
#define ED_OPT_TRLAN_NOFOLD   0x200 /* eigh: separate coefficient kernels on small grids       */
#define ED_OPT_NO_GRAPH       0x800 /* eigh: Krylov sweeps launched directly, not as hipGraphs  */
#define ED_OPT_TRLAN_NOLOCAL  0x1000 /* eigh: plain w = H v_j (no shifted three-term step)     */
#define ED_OPT_TRLAN_NOSOLO   0x2000 /* eigh: multi-kernel CGS also on sectors <= 2048 rows     */
#define ED_OPT_TRLAN_FULLUPD  0x4000 /* eigh: full CGS update every step (no local-only update) */
#define ED_OPT_STORED_EXACT 0x100000 /* stored H·v: the one-pass kernel (spMatVec_cc's per-row order,
                                        bit-identical) even where the two-segment form is built */
#define ED_OPT_NO_FUSED     0x400000 /* stored H·v: not the fused re-laid one-pass kernel (the
                                        two-segment form where built, else the one-pass one) */
#define ED_OPT_EIGH_NOHINT  0x800000 /* eigh: degeneracy screen from a pure hash start (no next
                                        Ritz vector mixed in) */
#define ED_OPT_EIGH_FULLPROBE 0x200000 /* eigh: no plain-Lanczos screen before the thick-restart
                                          degeneracy probe (every probe round runs it in full) */

/* status codes */
#define ED_OK              0
#define ED_ERR_ARG         1
#define ED_ERR_STATE       2
#define ED_ERR_HIP         3
#define ED_ERR_OOM         4
#define ED_ERR_UNSUPPORTED 5
#define ED_ERR_NOCONV      6 /* iterative solve did not converge */

/* ---------------------------------------------------------------- params
 * All arrays are C row-major over the MAXIMUM dimensions below; only the
 * leading [nspin][nspin][norb][norb][nbath] part is read.  Index i of a C array
 * here is Fortran index i+1 of the reference array.
 *   imphloc_*[ispin][jspin][iorb][jorb]      = impHloc(ispin+1,jspin+1,iorb+1,jorb+1)
 *   bath_e[ispin][iorb][k]                   = dmft_bath%e(ispin+1,iorb+1,k+1)
 *     (bath_type='hybrid': only iorb=0 is used, as size(e,2)=1)
 *   bath_v/u/d[ispin][iorb][k]               = dmft_bath%v/u/d(...)
 *   bath_h_*[ispin][jspin][iorb][jorb][k]    = dmft_bath%h(...)   (replica)
 *   bath_vr_*[k]                             = dmft_bath%vr(k+1)  (replica)
 */
typedef struct ed_params {
  int32_t norb, nspin, nbath;
  int32_t ed_mode;   /* ED_MODE_*  */
  int32_t bath_type; /* ED_BATH_*  */
  int32_t hfmode;    /* logical    */
  double uloc[3];
  double ust, jh, jx, jp, xmu;
  double imphloc_re[ED_MAX_NSPIN][ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NORB];
  double imphloc_im[ED_MAX_NSPIN][ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NORB];
  double bath_e[ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NBATH];
  double bath_v[ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NBATH];
  double bath_u[ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NBATH];
  double bath_d[ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NBATH];
  double bath_h_re[ED_MAX_NSPIN][ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NORB][ED_MAX_NBATH];
  double bath_h_im[ED_MAX_NSPIN][ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NORB][ED_MAX_NBATH];
  double bath_vr_re[ED_MAX_NBATH];
  double bath_vr_im[ED_MAX_NBATH];
  /* Jz_basis (ED_INPUT_VARS.f90:78, nonsu2 only): sectors are (n, twoJz) with
   * twoJz = twoSz + twoLz, twoLz = sum over levels of 2*Lzdiag(iorb) with
   * Lzdiag = [-1,+1,0] (ED_VARS_GLOBAL.f90:207) and iorb-1 = level mod Norb
   * (build_sector ED_SETUP.f90:940-965); q1 = n, q2 = twoJz.  H must conserve
   * Jz (replica bath with an Lz-basis Hloc): ed_sector_create checks it. */
  int32_t jz_basis;
  int32_t pad_;
} ed_params;

typedef struct ed_sector_info {
  int64_t dim;      /* getDim(isector)                                  */
  int64_t nnz;      /* stored elements incl. diagonal (0 for direct)    */
  int64_t padded;   /* SELL-64 slots actually stored (>= nnz - dim)     */
  int32_t ns;       /* levels per spin                                  */
  int32_t mode;     /* ED_MODE_*                                        */
  int32_t q1, q2;   /* (nup,ndw) | (sz,0) | (n,0) | (n,twoJz)           */
  int32_t flags;    /* ED_STORED|ED_DIRECT|ED_REAL as built             */
  int32_t kron;     /* 1 if the direct path uses the (DimUp x DimDw) form */
  int64_t dimup, dimdw;   /* factor dimensions (normal mode), else 0    */
  int64_t device_bytes;   /* device memory held by the sector           */
  int32_t packed;   /* 1 if stored H·v reads 32-bit {col|value index} words */
  int32_t npdict;   /* distinct off-diagonal values (packed dictionary)  */
  int64_t row0, nrows;    /* rows held: [row0, row0+nrows) (whole: 0, dim) */
  int32_t split;    /* 1 if the two-segment stored form is built (default stored H·v) */
  int32_t pad_;
  int64_t split_far;          /* cross-block elements (segment B)            */
  int64_t split_far_uniform;  /* of which stored once per 64-row slice (U)   */
  int64_t split_bytes;        /* bytes one two-segment launch reads of the re-laid matrix:
                                 4 * (A words + L words) + 8 * U entries + A slice pointers */
  int64_t split_list_bytes;   /* + segment B's work list and slice table       */
  int32_t fused;    /* 1 if the fused one-pass re-laid form is built (default stored H·v) */
  int32_t pad2_;
  int64_t fused_far;          /* cross-block elements                         */
  int64_t fused_far_uniform;  /* of which stored once per 64-row unit (U)     */
  int64_t fused_bytes;        /* bytes one fused launch reads of the re-laid matrix:
                                 4 * (A words + L words) + 8 * U entries + 40 * units */
} ed_sector_info;

typedef struct ed_sector ed_sector; /* opaque */

/* ------------------------------------------------------------ handle API */
/* Build the sector basis and (ED_STORED) the Hamiltonian on `device`.
 * q1,q2: (nup,ndw) for normal, (sz,-) for superc, (n,-) for nonsu2.
 * stream: NULL — the sector creates (and destroys) a private non-blocking
 * stream for its build and its synchronous entry points (eigh, lanczos, ...);
 * non-NULL — that stream is used instead and stays the caller's (it must
 * outlive the sector; a farm worker passes its own stream to every sector it
 * solves).  Do not pass the legacy default stream: it serialises with every
 * other stream of the device. */
int ed_sector_create(const ed_params* p, int32_t q1, int32_t q2, int32_t flags,
                     int32_t device, void* stream, ed_sector** out);
/* The reference's MPI row split of one sector (build_Hv_sector with
 * MpiStatus, ED_HAMILTONIAN.f90:55-62; spMatVec_mpi_cc STORED_HxV.f90:147-197):
 * build only rows [row0, row0+nrows) of H (ED_STORED, or ED_DIRECT generic).
 * ed_sector_hxv_dev[_path] then takes the WHOLE sector vector v (the
 * Allgatherv result) and writes the nrows local entries of Hv; columns stay
 * global.  Lanczos/eigh/apply_op refuse such a sector (ED_ERR_UNSUPPORTED):
 * the distributed recurrence runs on the host side (edgpu.dist). */
int ed_sector_create_rows(const ed_params* p, int32_t q1, int32_t q2, int32_t flags, int64_t row0,
                          int64_t nrows, int32_t device, void* stream, ed_sector** out);
int ed_sector_destroy(ed_sector* s);
/* Select kernel alternatives (ED_OPT_* bit set, replaces the previous set). */
int ed_sector_set_options(ed_sector* s, int32_t opts);
int ed_sector_get_info(const ed_sector* s, ed_sector_info* info);

/* H·v on device pointers (async on `stream`).  vtype: 0 = real(8) vectors,
 * 1 = complex(8) interleaved vectors.  hv is overwritten (not accumulated),
 * as spMatVec_cc does (Hv=zero first, STORED_HxV.f90:137). */
int ed_sector_hxv_dev(ed_sector* s, int32_t vtype, const void* v, void* hv, void* stream);
/* Same, forcing the matrix-free kernel even on a stored sector (1) or the
 * stored kernel (0). -1 = default for the sector. */
int ed_sector_hxv_dev_path(ed_sector* s, int32_t path, int32_t vtype, const void* v,
                           void* hv, void* stream);
/* Columns the held rows refer to (the halo of a row-split sector,
 * ed_sector_create_rows): mask_dev[(dim+31)/32] (device, zeroed here) gets bit
 * c set for every column c of an off-diagonal element of the held rows.
 * Async on `stream`.  edgpu.dist exchanges only these entries of the vector
 * instead of the reference's whole-vector Allgatherv (STORED_HxV.f90:175-189). */
int ed_sector_col_mask(const ed_sector* s, uint32_t* mask_dev, void* stream);
/* Host-pointer H·v (synchronous, complex(8) vectors of length nloc = dim). */
int ed_sector_hxv(ed_sector* s, int32_t nloc, const double* v, double* hv);

/* H%map(1:dim): the Fock states of the sector in reference order (uint32). */
int ed_sector_map(const ed_sector* s, uint32_t* map_host);
/* Dump the stored H in reference row order (diagonal first, then off-diagonal
 * elements in insertion order).  rowptr[dim+1], cols[nnz] are 0-based;
 * vals is complex interleaved (2*nnz doubles).  Requires ED_STORED. */
int ed_sector_dump_csr(const ed_sector* s, int64_t* rowptr, int32_t* cols, double* vals);

/* Read-only view of the device SELL-64 arrays of a stored sector (for
 * inspection / kernel experiments).  Entry k of row r lives at
 * sptr[r/64] + 64*k + r%64; the diagonal is separate.  vals/diag are real(8)
 * when value_bytes == 8, complex(8) interleaved when 16. */
typedef struct ed_sell_view {
  int64_t dim, nslice, slots;
  int32_t value_bytes, pad;
  const void* diag;
  const int64_t* sptr;
  const int32_t* cols;
  const void* vals;
  const uint16_t* rowcnt;
} ed_sell_view;
int ed_sector_sell_view(const ed_sector* s, ed_sell_view* view);

/* Device-resident plain Lanczos (3-term recurrence, no reorthogonalisation).
 * v0: host start vector (vtype as above) of length dim, or NULL for the
 * deterministic default start vector.  Outputs on the host. */
int ed_sector_lanc_tridiag(ed_sector* s, int32_t vtype, const void* v0, int32_t nitermax,
                           double threshold, double* alfa, double* beta, int32_t* nlanc);
/* Ground state: returns egs (lowest Ritz value) and, if vect != NULL, the
 * normalised Ritz vector (host or device pointer, vtype).  ncheck as
 * lanczos_plain_c. */
int ed_sector_lanc_eigh(ed_sector* s, int32_t vtype, const void* v0, int32_t nitermax,
                        double threshold, int32_t ncheck, double* egs, void* vect,
                        int32_t* nlanc);
/* Diagnostic: the Lanczos recurrence a run with (vtype, path) would use —
 * persistent one-workgroup mode 0 (stored, L2), 1 (Kronecker tables in LDS),
 * 2 (stored matrix in registers), 3 (its matrix-free twin), 4 (Kronecker
 * register layout) or -1 (graph-captured multi-kernel), under the sector's
 * ED_OPT_* options. */
int ed_sector_lanc_mode(ed_sector* s, int32_t vtype, int32_t path);
/* Lowest `nev` eigenpairs by thick-restart Lanczos with full (CGS2)
 * reorthogonalisation, Krylov basis of `ncv` vectors resident in HBM: the
 * device replacement of SciFortran's ARPACK sp_eigh (ED_DIAG.f90:145-167,
 * which="SR", Nblock=ncv, Nitermax=maxit restarts, tol as ARPACK:
 * |r_i| <= tol*max(eps^(2/3),|theta_i|)).  v0: host start vector or NULL.
 * evals[nev] ascending; evecs (host or device pointer, dim x nev
 * column-major, vtype) or NULL.
 * nconv: converged pairs; nhv: H·v products used.  ncv <= 64. */
int ed_sector_eigh(ed_sector* s, int32_t vtype, int32_t nev, int32_t ncv, int32_t maxit, double tol,
                   const void* v0, double* evals, void* evecs, int32_t* nconv, int32_t* nhv);
/* ed_sector_eigh (real vectors) for n stored sectors at once, the same
 * algorithm and options per sector: sectors of up to 2,640 rows run their
 * restart cycles and degeneracy-screen chunks as one workgroup each in a
 * shared launch (one launch and one host round trip per cycle for all of
 * them); larger ones run in lockstep, every kernel of a Krylov step carrying
 * that step of all of them; sectors the batch cannot take or finish are
 * solved by ed_sector_eigh's path afterwards.  The farm's replacement of
 * ED_DIAG.f90:71-249's loop over the sectors' sp_eigh calls.  maxit[i]:
 * sector i's Nitermax; v0[i] (host, or NULL / v0 NULL: the default start),
 * evals[i*nev + k], evecs[i] (host or device, dim x nev, or NULL), nconv[i],
 * nhv[i]; *nbatched: sectors finished inside the batch (or NULL); flags:
 * ED_BATCH_NO_FALLBACK leaves the others to the caller (their nconv[i] = -1,
 * e.g. to solve them on several threads); stream: the launches' stream
 * (NULL: the first sector's). */
#define ED_BATCH_NO_FALLBACK 0x1
int ed_sectors_eigh_batch(ed_sector* const* secs, int32_t n, int32_t nev, int32_t ncv, const int32_t* maxit,
                          double tol, const double* const* v0, double* evals, void* const* evecs,
                          int32_t* nconv, int32_t* nhv, int32_t* nbatched, int32_t flags, void* stream);
/* Fixed-length Lanczos on device pointers for benchmarking: runs exactly
 * `niter` iterations (no convergence test) from device vector v0 and writes
 * alfa/beta (host).  Returns the elapsed device time in ms in *ms (or NULL). */
int ed_sector_lanc_run(ed_sector* s, int32_t vtype, const void* v0_dev, int32_t niter,
                       double* alfa, double* beta, float* ms, void* stream);

/* Within-sector multi-GPU H·v (replaces the reference's MPI
 * row split + Allgatherv, ED_HAMILTONIAN.f90:55-62, STORED_HxV.f90:147-197)
 * for sectors built with ED_DIRECT that have the Kronecker form (info.kron):
 * H = D + Hup(x)1 + 1(x)Hdw on the DimDw x DimUp view of v.
 *   kron_rows: y[r][:] = D[w0+r][:] .* x[r][:] + Hup x[r][:]      (r < nw)
 *              x, y: the nw x DimUp row block of down rows [w0, w0+nw)
 *   kron_cols: yz[:][c] (+)= Hdw z[:][c]                           (c < nu)
 *              z, yz: the DimDw x nu strip of up columns [u0, u0+nu),
 *              row-major (c fastest); accumulate = 1 adds into yz
 * H v = rows(x) + cols(strip(x)) regathered: two all-to-alls per H·v, whose
 * row blocks are already the strip layout (edgpu.dist).  Device pointers,
 * async on `stream`. */
int ed_sector_kron_rows(ed_sector* s, int32_t vtype, int64_t w0, int64_t nw, const void* x, void* y,
                        void* stream);
int ed_sector_kron_cols(ed_sector* s, int32_t vtype, int64_t u0, int64_t nu, const void* z, void* yz,
                        int32_t accumulate, void* stream);

/* Green's-function seed (ED_GF_NORMAL.f90:159-174 / :216-229):
 *   dst(j) = sg * src(m)  for every basis state m of `src` with the level
 *   free (op = 1, c^+) or occupied (op = 0, c), |j> = op_level |m>,
 *   sg the Jordan-Wigner sign of c / cdg (ED_SETUP.f90:1080-1106).
 * `level` is the 0-based bit (Fortran position - 1).  dst is zeroed first.
 * Device pointers, async on `stream`; both sectors on the same device. */
int ed_sector_apply_op(const ed_sector* src, const ed_sector* dst, int32_t op, int32_t level,
                       int32_t vtype, const void* src_vec, void* dst_vec, void* stream);
/* Accumulating form for the mixed nonSU2 seeds (ED_GF_NONSU2.f90:571-595,
 * 739-763): dst(j) += (coef_re + i coef_im) * sg * src(m); dst is NOT zeroed.
 * vtype must be 1 (complex) when coef_im != 0. */
int ed_sector_apply_op_acc(const ed_sector* src, const ed_sector* dst, int32_t op, int32_t level,
                           double coef_re, double coef_im, int32_t vtype, const void* src_vec,
                           void* dst_vec, void* stream);
/* sp_lanc_tridiag from a device start vector (not modified). */
/* v0_dev must be complete on entry (synchronise the stream that wrote it). */
int ed_sector_lanc_tridiag_dev(ed_sector* s, int32_t vtype, const void* v0_dev, int32_t nitermax,
                               double threshold, double* alfa, double* beta, int32_t* nlanc);
/* sp_lanc_tridiag for nseed device start vectors (v0_dev: nseed x dim,
 * contiguous, not modified) on the same sector — the Green's-function seeds
 * of one target sector (ED_GF_NORMAL.f90:180-193, ED_GF_NONSU2.f90:343-886).
 * Sectors that run the persistent one-workgroup recurrence take all seeds in
 * one launch, one workgroup per seed; alfa/beta/nlanc: nseed x nitermax /
 * nseed, each as ed_sector_lanc_tridiag. */
int ed_sector_lanc_tridiag_batch(ed_sector* s, int32_t vtype, int32_t nseed, const void* v0_dev,
                                 int32_t nitermax, double threshold, double* alfa, double* beta,
                                 int32_t* nlanc);
/* GF poles of one continued fraction (host, O(n^2)): E[n] ascending eigenvalues
 * of tridiag(alfa[0:n], beta[1:n]), z2[n] the squared first components of
 * their eigenvectors and (z1 != NULL) the first components themselves, Z(1,j).
 * Replaces tql2 in add_to_lanczos_gf_nonsu2 (ED_GF_NONSU2.f90:936;
 * ED_GF_SHARED.f90:76-214) and eigh in add_to_lanczos_gf_normal
 * (ED_GF_NORMAL.f90:612-618). */
int ed_tridiag_poles(int32_t n, const double* alfa, const double* beta, double* E, double* z2, double* z1);
/* Pole sums of nfrac continued fractions into device-resident G, in list
 * order — the inner loops of add_to_lanczos_gf_normal (ED_GF_NORMAL.f90:
 * 620-631) and add_to_lanczos_gf_nonsu2 (ED_GF_NONSU2.f90:936-950): fraction
 * f has npole[f] poles (E, z = Z(1,j): concatenated over fractions, host
 * arrays), weight pesoBZ = peso_bz[2f] + i peso_bz[2f+1], energy Ei[f], sign
 * isign[f] = +-1 and target component comp[f]; for every frequency
 *   gm[comp][i] += (pesoBZ*z_j)*z_j / (i*wm[i] - isign*(E_j - Ei))
 *   gr[comp][i] += (pesoBZ*z_j)*z_j / (wr[i] + i*eps - isign*(E_j - Ei))
 * pole by pole (the reference's addition order).  gm (ncomp x lmats), gr
 * (ncomp x lreal): complex(8) device arrays; wm[lmats], wr[lreal]: device.
 * Synchronous on `stream` (the host pole data is staged). */
int ed_gf_add_poles(int32_t nfrac, const int32_t* npole, const double* E, const double* z, const double* peso_bz,
                    const double* Ei, const int32_t* isign, const int32_t* comp, const double* wm, int32_t lmats,
                    const double* wr, int32_t lreal, double eps, double* gm, double* gr, void* stream);

/* ------------------------------------------------------ reference-style API */
int ed_gpu_init(const ed_params* p);          /* ed_init_solver parameter hand-over */
int ed_gpu_set_device(int32_t device);
int ed_gpu_build_sector(int32_t q1, int32_t q2, int32_t flags, int64_t* dim);
int ed_gpu_vecdim(int32_t* vecdim);           /* vecDim_Hv_sector of the current sector */
/* cc_sparse_HxV(Nloc,v,Hv): Nloc by reference, complex(8) host arrays. */
int ed_gpu_hxv(const int32_t* nloc, const double* v, double* hv);
/* MPI variant of the current sector (MpiStatus=T in build_Hv_sector,
 * ED_HAMILTONIAN.f90:55-62, 85-101): this rank holds rows [row0, row0+nrows)
 * of H (nrows may be 0 when dim < MpiSize); vecDim_Hv_sector is then nrows. */
int ed_gpu_build_sector_rows(int32_t q1, int32_t q2, int32_t flags, int64_t row0, int64_t nrows,
                             int64_t* dim);
/* The reference's row split (ED_HAMILTONIAN.f90:55-62): MpiQ = dim/size, the
 * last rank also takes mod(dim,size); row0 = MpiIshift (0-based MpiIstart). */
int ed_gpu_mpi_split(int64_t dim, int32_t rank, int32_t size, int64_t* row0, int64_t* nrows);
/* spMatVec_mpi_cc (ED_HAMILTONIAN_STORED_HxV.f90:147-197) after its
 * MPI_Allgatherv: vin is the whole sector vector (dim, complex(8)), hv the
 * nloc = nrows local entries.  The Allgatherv itself stays in the caller's MPI
 * (the Fortran shim's gpuMatVec_mpi_cc).  Summation: every local row in the
 * reference's serial element order (spMatVec_cc); the reference's MPI kernel
 * adds the local-column elements first, so the two differ by rounding. */
int ed_gpu_hxv_mpi(const int32_t* nloc, const double* vin, double* hv);
int ed_gpu_dump_csr(int64_t* rowptr, int32_t* cols, double* vals);
int ed_gpu_lanc_eigh(int32_t nitermax, double threshold, int32_t ncheck, double* egs,
                     double* vect, int32_t* nlanc);
/* sp_eigh(spHtimesV_cc, eig_values, eig_basis, Nblock, Nitermax, tol)
 * (ED_DIAG.f90:145-167, ARPACK which="SR"): device thick-restart Lanczos on
 * the current sector, complex(8) vectors.  v0 (dim, complex) or NULL;
 * evals[neigen] ascending; evecs complex(8) (dim x neigen, column-major) or
 * NULL; nconv converged pairs. */
int ed_gpu_eigh(int32_t neigen, int32_t nblock, int32_t nitermax, double tol, const double* v0,
                double* evals, double* evecs, int32_t* nconv);
int ed_gpu_lanc_tridiag(const double* v0, int32_t nitermax, double threshold,
                        double* alfa, double* beta, int32_t* nlanc);
int ed_gpu_delete_sector(void);
int ed_gpu_finalize(void);
const char* ed_gpu_last_error(void);
int ed_gpu_current_sector(ed_sector** out);   /* handle of the current sector */

#ifdef __cplusplus
}
#endif
#endif /* ED_GPU_H */
