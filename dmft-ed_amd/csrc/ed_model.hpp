// ed_model.hpp — device-side model constants and the row element generator.
//
// The generator is the single source of matrix elements for every device
// path (stored-H builder, matrix-free H·v, GF seeds): for a basis state m it
// produces the row of H in the *stored* convention of the reference,
//   H(i,j) = conj(coeff) * sg,   |k_j> = op |m_i>          (ED_HAMILTONIAN/stored/*.f90)
// in the exact insertion order of ed_buildH_c, so that the stored matrix
// reproduces spH0 (ED_SPARSE_MATRIX row-of-arrays) element by element.
// By hermiticity the same row drives the gather-form matrix-free kernel,
//   Hv(i) = sum_j H(i,j) v(j),
// which replaces the reference's scatter loop (ED_HAMILTONIAN_DIRECT_HxV.f90:68-89).
//
// FP contraction is disabled in every TU that includes this file (-ffp-contract=off):
// the diagonal is accumulated one IEEE op at a time in reference order, which
// makes stored values bit-identical to the reference expression order.
#pragma once
#include <stdint.h>

#include "../../include/ed_gpu.h"

#ifndef ED_HD
#define ED_HD __host__ __device__ __forceinline__
#endif

namespace edg {

struct EdModel {
  int32_t ns, norb, nbath, nspin, S, mode, bath, ne, jhflag, hfmode;
  int32_t jz;                 // nonsu2 Jz_basis sectors (n, twoJz)
  int32_t lz2[ED_MAX_NS];     // 2*Lzdiag(iorb) of level l, iorb-1 = l mod Norb (ED_SETUP.f90:954)
  int32_t stride[ED_MAX_NORB][ED_MAX_NBATH];  // getBathStride, 0-based bit
  double hloc_re[ED_MAX_NSPIN][ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NORB];
  double hloc_im[ED_MAX_NSPIN][ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NORB];
  double uloc[3], ust, jh, jx, jp, xmu;
  double e[ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NBATH];
  double u[ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NBATH];
  double d[ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NBATH];
  double hyb_re[ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NBATH];  // diag_hybr (STORED_HxV.f90:58-70)
  double hyb_im[ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NBATH];
  double hb_re[ED_MAX_NSPIN][ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NORB][ED_MAX_NBATH];
  double hb_im[ED_MAX_NSPIN][ED_MAX_NSPIN][ED_MAX_NORB][ED_MAX_NORB][ED_MAX_NBATH];
};

// Host: fill the model from the C-ABI params.  Returns 0 or an ED_ERR_* code.
// ed_setup_dimensions ED_SETUP.f90:96-111, getBathStride ED_SETUP.f90:448-465,
// Jhflag ED_SETUP.f90:289-290.
inline int model_from_params(const ed_params* p, EdModel* M) {
  if (!p) return ED_ERR_ARG;
  if (p->norb < 1 || p->norb > ED_MAX_NORB || p->nspin < 1 || p->nspin > ED_MAX_NSPIN ||
      p->nbath < 0 || p->nbath > ED_MAX_NBATH)
    return ED_ERR_ARG;
  if (p->ed_mode < 0 || p->ed_mode > 2 || p->bath_type < 0 || p->bath_type > 2) return ED_ERR_ARG;
  if (p->ed_mode == ED_MODE_NONSU2 && p->nspin != 2) return ED_ERR_ARG;  // ed_checks_global
  if (p->ed_mode == ED_MODE_SUPERC && p->nspin != 1) return ED_ERR_ARG;
  *M = EdModel{};
  M->norb = p->norb; M->nbath = p->nbath; M->nspin = p->nspin; M->S = p->nspin - 1;
  M->mode = p->ed_mode; M->bath = p->bath_type; M->hfmode = p->hfmode ? 1 : 0;
  M->ns = (p->bath_type == ED_BATH_HYBRID) ? p->nbath + p->norb : (p->nbath + 1) * p->norb;
  if (M->ns > ED_MAX_NS) return ED_ERR_UNSUPPORTED;
  M->ne = (p->bath_type == ED_BATH_HYBRID) ? 1 : p->norb;
  M->jhflag = (p->norb > 1 && (p->jx != 0.0 || p->jp != 0.0)) ? 1 : 0;
  if (p->jz_basis) {
    // Lzdiag = [-1,+1,0] (ED_VARS_GLOBAL.f90:207) is defined for Norb <= 3 and
    // the level -> orbital map of build_sector assumes Ns = Norb*(Nbath+1)
    if (p->ed_mode != ED_MODE_NONSU2 || p->norb > 3 || p->bath_type == ED_BATH_HYBRID)
      return ED_ERR_UNSUPPORTED;
    static const int lzd[3] = {-1, +1, 0};
    M->jz = 1;
    for (int l = 0; l < M->ns; l++) M->lz2[l] = 2 * lzd[l % p->norb];
  }
  for (int k = 0; k < p->nbath; k++)
    for (int o = 0; o < p->norb; o++) {
      int lev;
      if (p->bath_type == ED_BATH_HYBRID) lev = p->norb + (k + 1);
      else if (p->bath_type == ED_BATH_REPLICA) lev = (o + 1) + (k + 1) * p->norb;
      else lev = p->norb + o * p->nbath + (k + 1);
      M->stride[o][k] = lev - 1;
    }
  for (int a = 0; a < ED_MAX_NSPIN; a++)
    for (int b = 0; b < ED_MAX_NSPIN; b++)
      for (int c = 0; c < ED_MAX_NORB; c++)
        for (int d = 0; d < ED_MAX_NORB; d++) {
          M->hloc_re[a][b][c][d] = p->imphloc_re[a][b][c][d];
          M->hloc_im[a][b][c][d] = p->imphloc_im[a][b][c][d];
          for (int k = 0; k < ED_MAX_NBATH; k++) {
            M->hb_re[a][b][c][d][k] = p->bath_h_re[a][b][c][d][k];
            M->hb_im[a][b][c][d][k] = p->bath_h_im[a][b][c][d][k];
          }
        }
  for (int i = 0; i < 3; i++) M->uloc[i] = p->uloc[i];
  M->ust = p->ust; M->jh = p->jh; M->jx = p->jx; M->jp = p->jp; M->xmu = p->xmu;
  for (int s = 0; s < ED_MAX_NSPIN; s++)
    for (int o = 0; o < ED_MAX_NORB; o++)
      for (int k = 0; k < ED_MAX_NBATH; k++) {
        M->e[s][o][k] = p->bath_e[s][o][k];
        M->u[s][o][k] = p->bath_u[s][o][k];
        M->d[s][o][k] = p->bath_d[s][o][k];
        if (p->bath_type != ED_BATH_REPLICA) {
          M->hyb_re[s][o][k] = p->bath_v[s][o][k];
          M->hyb_im[s][o][k] = 0.0;
        } else {
          M->hyb_re[s][o][k] = p->bath_vr_re[k];
          M->hyb_im[s][o][k] = p->bath_vr_im[k];
        }
      }
  return ED_OK;
}

// True when every coefficient that can enter H is real.
inline bool model_is_real(const EdModel& M) {
  for (int a = 0; a < ED_MAX_NSPIN; a++)
    for (int b = 0; b < ED_MAX_NSPIN; b++)
      for (int c = 0; c < ED_MAX_NORB; c++)
        for (int d = 0; d < ED_MAX_NORB; d++) {
          if (M.hloc_im[a][b][c][d] != 0.0) return false;
          for (int k = 0; k < ED_MAX_NBATH; k++)
            if (M.hb_im[a][b][c][d][k] != 0.0) return false;
        }
  for (int s = 0; s < ED_MAX_NSPIN; s++)
    for (int o = 0; o < ED_MAX_NORB; o++)
      for (int k = 0; k < ED_MAX_NBATH; k++)
        if (M.hyb_im[s][o][k] != 0.0) return false;
  return true;
}

ED_HD int bit(uint32_t x, int b) { return (int)((x >> b) & 1u); }

// c / cdg (ED_SETUP.f90:1080-1106): Jordan-Wigner sign = (-1)^popcount(bits below b).
ED_HD double jw_sign(uint32_t in, int b) {
  uint32_t below = (b == 0) ? 0u : (in & ((1u << b) - 1u));
  return (__builtin_popcount(below) & 1) ? -1.0 : 1.0;
}

// Local interaction on the diagonal, stored/Hint.f90:11-49 (= direct/HxVint.f90:1-47).
// upbits/dwbits: impurity occupations n_{o,up} = bit o of upbits, n_{o,dw} = bit o of dwbits.
ED_HD double hint_value(const EdModel& M, uint32_t upbits, uint32_t dwbits) {
  const int norb = M.norb;
#define nup(o) ((double)bit(upbits, (o)))
#define ndw(o) ((double)bit(dwbits, (o)))
  double h = 0.0;
  for (int o = 0; o < norb; o++) h = h + (M.uloc[o] * nup(o)) * ndw(o);
  if (norb > 1) {
    for (int o = 0; o < norb; o++)
      for (int q = o + 1; q < norb; q++) h = h + M.ust * (nup(o) * ndw(q) + nup(q) * ndw(o));
    for (int o = 0; o < norb; o++)
      for (int q = o + 1; q < norb; q++)
        h = h + (M.ust - M.jh) * (nup(o) * nup(q) + ndw(o) * ndw(q));
  }
  if (M.hfmode) {
    for (int o = 0; o < norb; o++) h = (h - (0.5 * M.uloc[o]) * (nup(o) + ndw(o))) + 0.25 * M.uloc[o];
    if (norb > 1)
      for (int o = 0; o < norb; o++)
        for (int q = o + 1; q < norb; q++) {
          double nn = ((nup(o) + ndw(o)) + nup(q)) + ndw(q);
          h = (h - (0.5 * M.ust) * nn) + 0.25 * M.ust;
          h = (h - (0.5 * (M.ust - M.jh)) * nn) + 0.25 * (M.ust - M.jh);
        }
  }
#undef nup
#undef ndw
  return h;
}

// ---------------------------------------------------------------- generator
// Acc must provide:
//   void diag(double re, double im);                 // once, first
//   void off(uint32_t k, double re, double im);      // off-diagonal, in order
// `ValuesOnly` accs may ignore arguments; the compiler removes dead math.
// The diagonal element of the row of state m (reference order, see gen_row).
ED_HD void gen_diag(const EdModel& M, uint32_t m, double* dre, double* dim_) {
  const int ns = M.ns, norb = M.norb, nbath = M.nbath, S = M.S;
  // nup(iorb)/ndw(iorb) of the reference, evaluated on the fly (no local arrays:
  // dynamically indexed arrays would spill to scratch on the GPU)
#define nup(o) ((double)bit(m, (o)))
#define ndw(o) ((double)bit(m, (o) + ns))
  // ---- diagonal: stored/Himp.f90:11-16, merged with Hint.f90:11-49 and
  //      Hbath.f90:13-27 / :33-40 (sp_insert_element adds into the first slot).
  double dr = 0.0, di = 0.0;
  for (int o = 0; o < norb; o++) {
    dr = dr + M.hloc_re[0][0][o][o] * nup(o);
    di = di + M.hloc_im[0][0][o][o] * nup(o);
    dr = dr + M.hloc_re[S][S][o][o] * ndw(o);
    di = di + M.hloc_im[S][S][o][o] * ndw(o);
    dr = dr - M.xmu * (nup(o) + ndw(o));
  }
  {
    double h = hint_value(M, m, m >> ns);
    dr = dr + h;
    di = di + 0.0;
  }
  if (M.bath != ED_BATH_REPLICA) {
    double h = 0.0;
    for (int o = 0; o < M.ne; o++)
      for (int k = 0; k < nbath; k++) {
        int a = M.stride[o][k];
        h = h + M.e[0][o][k] * (double)bit(m, a);
        h = h + M.e[S][o][k] * (double)bit(m, a + ns);
      }
    dr = dr + h;
    di = di + 0.0;
  } else {
    double hr = 0.0, hi = 0.0;
    for (int k = 0; k < nbath; k++)
      for (int o = 0; o < norb; o++) {
        int a = M.stride[o][k];
        double nu = (double)bit(m, a), nd = (double)bit(m, a + ns);
        hr = hr + M.hb_re[0][0][o][o][k] * nu;
        hi = hi + M.hb_im[0][0][o][o][k] * nu;
        hr = hr + M.hb_re[S][S][o][o][k] * nd;
        hi = hi + M.hb_im[S][S][o][o][k] * nd;
      }
    dr = dr + hr;
    di = di + hi;
  }
  *dre = dr;
  *dim_ = di;
#undef nup
#undef ndw
}

template <class Acc>
ED_HD void gen_row(const EdModel& M, uint32_t m, Acc& acc) {
  const int norb = M.norb, nbath = M.nbath, S = M.S, ns = M.ns;
  {
    double dr, di;
    gen_diag(M, m, &dr, &di);
    acc.diag(dr, di);
  }

  // ---- stored/Himp.f90:27-72 same-spin impurity hops, value conj(h)*sg1*sg2
  for (int io = 0; io < norb; io++)
    for (int jo = 0; jo < norb; jo++) {
      {
        double hr = M.hloc_re[0][0][io][jo], hi = M.hloc_im[0][0][io][jo];
        if ((hr != 0.0 || hi != 0.0) && bit(m, jo) == 1 && bit(m, io) == 0) {
          double s = jw_sign(m, jo);
          uint32_t k1 = m & ~(1u << jo);
          double s2 = jw_sign(k1, io);
          acc.off(k1 | (1u << io), (hr * s) * s2, (-hi * s) * s2);
        }
      }
      {
        double hr = M.hloc_re[S][S][io][jo], hi = M.hloc_im[S][S][io][jo];
        int a = io + ns, b = jo + ns;
        if ((hr != 0.0 || hi != 0.0) && bit(m, b) == 1 && bit(m, a) == 0) {
          double s = jw_sign(m, b);
          uint32_t k1 = m & ~(1u << b);
          double s2 = jw_sign(k1, a);
          acc.off(k1 | (1u << a), (hr * s) * s2, (-hi * s) * s2);
        }
      }
    }
  // ---- stored/Himp.f90:74-104 nonSU2 spin-flip impHloc
  if (M.mode == ED_MODE_NONSU2) {
    for (int is = 0; is < 2; is++) {
      int js = 1 - is;
      for (int io = 0; io < norb; io++)
        for (int jo = 0; jo < norb; jo++) {
          double hr = M.hloc_re[is][js][io][jo], hi = M.hloc_im[is][js][io][jo];
          int a = io + is * ns, b = jo + js * ns;
          if ((hr != 0.0 || hi != 0.0) && bit(m, b) == 1 && bit(m, a) == 0) {
            double s = jw_sign(m, b);
            uint32_t k1 = m & ~(1u << b);
            double s2 = jw_sign(k1, a);
            acc.off(k1 | (1u << a), (hr * s) * s2, (-hi * s) * s2);
          }
        }
    }
  }
  // ---- stored/Hint.f90:60-123 spin exchange and pair hopping
  if (norb > 1 && M.jhflag) {
    for (int io = 0; io < norb; io++)
      for (int jo = 0; jo < norb; jo++)
        if (io != jo && bit(m, jo) == 1 && bit(m, io + ns) == 1 && bit(m, jo + ns) == 0 &&
            bit(m, io) == 0) {
          double s1 = jw_sign(m, jo);
          uint32_t k1 = m & ~(1u << jo);
          double s2 = jw_sign(k1, io + ns);
          uint32_t k2 = k1 & ~(1u << (io + ns));
          double s3 = jw_sign(k2, jo + ns);
          uint32_t k3 = k2 | (1u << (jo + ns));
          double s4 = jw_sign(k3, io);
          acc.off(k3 | (1u << io), (((M.jx * s1) * s2) * s3) * s4, 0.0);
        }
    for (int io = 0; io < norb; io++)
      for (int jo = 0; jo < norb; jo++)
        if (io != jo && bit(m, jo) == 1 && bit(m, jo + ns) == 1 && bit(m, io + ns) == 0 &&
            bit(m, io) == 0) {
          double s1 = jw_sign(m, jo);
          uint32_t k1 = m & ~(1u << jo);
          double s2 = jw_sign(k1, jo + ns);
          uint32_t k2 = k1 & ~(1u << (jo + ns));
          double s3 = jw_sign(k2, io + ns);
          uint32_t k3 = k2 | (1u << (io + ns));
          double s4 = jw_sign(k3, io);
          acc.off(k3 | (1u << io), (((M.jp * s1) * s2) * s3) * s4, 0.0);
        }
  }
  // ---- stored/Hbath.f90:52-135 replica bath hops (same spin, then nonSU2 flips)
  if (M.bath == ED_BATH_REPLICA) {
    for (int k = 0; k < nbath; k++)
      for (int io = 0; io < norb; io++)
        for (int jo = 0; jo < norb; jo++)
          for (int sp = 0; sp < 2; sp++) {
            int ss = sp == 0 ? 0 : S;
            double hr = M.hb_re[ss][ss][io][jo][k], hi = M.hb_im[ss][ss][io][jo][k];
            int a = M.stride[io][k] + sp * ns, b = M.stride[jo][k] + sp * ns;
            if ((hr != 0.0 || hi != 0.0) && bit(m, b) == 1 && bit(m, a) == 0) {
              double s = jw_sign(m, b);
              uint32_t k1 = m & ~(1u << b);
              double s2 = jw_sign(k1, a);
              acc.off(k1 | (1u << a), (hr * s) * s2, (-hi * s) * s2);
            }
          }
    if (M.mode == ED_MODE_NONSU2) {
      for (int k = 0; k < nbath; k++)
        for (int is = 0; is < 2; is++) {
          int js = 1 - is;
          for (int io = 0; io < norb; io++)
            for (int jo = 0; jo < norb; jo++) {
              double hr = M.hb_re[is][js][io][jo][k], hi = M.hb_im[is][js][io][jo][k];
              int a = M.stride[io][k] + is * ns, b = M.stride[jo][k] + js * ns;
              if ((hr != 0.0 || hi != 0.0) && bit(m, b) == 1 && bit(m, a) == 0) {
                double s = jw_sign(m, b);
                uint32_t k1 = m & ~(1u << b);
                double s2 = jw_sign(k1, a);
                acc.off(k1 | (1u << a), (hr * s) * s2, (-hi * s) * s2);
              }
            }
        }
    }
  }
  // ---- stored/Hbath.f90:142-178 superconducting pair terms
  if (M.mode == ED_MODE_SUPERC) {
    for (int o = 0; o < M.ne; o++)
      for (int k = 0; k < nbath; k++) {
        int ms = M.stride[o][k];
        double dd = M.d[0][o][k];
        if (dd != 0.0 && bit(m, ms) == 1 && bit(m, ms + ns) == 1) {
          double s1 = jw_sign(m, ms);
          uint32_t k1 = m & ~(1u << ms);
          double s2 = jw_sign(k1, ms + ns);
          acc.off(k1 & ~(1u << (ms + ns)), (dd * s1) * s2, 0.0);
        }
        if (dd != 0.0 && bit(m, ms) == 0 && bit(m, ms + ns) == 0) {
          double s1 = jw_sign(m, ms + ns);
          uint32_t k1 = m | (1u << (ms + ns));
          double s2 = jw_sign(k1, ms);
          acc.off(k1 | (1u << ms), (dd * s1) * s2, 0.0);
        }
      }
  }
  // ---- stored/Himp_bath.f90:10-67 spin-conserving hybridisation
  for (int o = 0; o < norb; o++)
    for (int k = 0; k < nbath; k++) {
      int ms = M.stride[o][k];
      for (int sp = 0; sp < 2; sp++) {
        int ss = sp == 0 ? 0 : S;
        double hr = M.hyb_re[ss][o][k], hi = M.hyb_im[ss][o][k];
        bool nz = (hr != 0.0 || hi != 0.0);
        int a = o + sp * ns, b = ms + sp * ns;  // impurity level, bath level
        if (nz && bit(m, a) == 1 && bit(m, b) == 0) {
          double s = jw_sign(m, a);
          uint32_t k1 = m & ~(1u << a);
          double s2 = jw_sign(k1, b);
          acc.off(k1 | (1u << b), (hr * s) * s2, (-hi * s) * s2);
        }
        if (nz && bit(m, a) == 0 && bit(m, b) == 1) {
          double s = jw_sign(m, b);
          uint32_t k1 = m & ~(1u << b);
          double s2 = jw_sign(k1, a);
          acc.off(k1 | (1u << a), (hr * s) * s2, (-hi * s) * s2);
        }
      }
    }
  // ---- stored/Himp_bath.f90:70-128 nonSU2 spin-flip hybridisation (no u/=0 test)
  if (M.mode == ED_MODE_NONSU2 && M.bath != ED_BATH_REPLICA) {
    for (int o = 0; o < norb; o++)
      for (int k = 0; k < nbath; k++) {
        int ms = M.stride[o][k];
        double uu = M.u[0][o][k], ud = M.u[S][o][k];
        // IMP UP <--> BATH DW
        if (bit(m, o) == 1 && bit(m, ms + ns) == 0) {
          double s = jw_sign(m, o);
          uint32_t k1 = m & ~(1u << o);
          double s2 = jw_sign(k1, ms + ns);
          acc.off(k1 | (1u << (ms + ns)), (uu * s) * s2, 0.0);
        }
        if (bit(m, o) == 0 && bit(m, ms + ns) == 1) {
          double s = jw_sign(m, ms + ns);
          uint32_t k1 = m & ~(1u << (ms + ns));
          double s2 = jw_sign(k1, o);
          acc.off(k1 | (1u << o), (uu * s) * s2, 0.0);
        }
        // IMP DW <--> BATH UP
        if (bit(m, o + ns) == 1 && bit(m, ms) == 0) {
          double s = jw_sign(m, o + ns);
          uint32_t k1 = m & ~(1u << (o + ns));
          double s2 = jw_sign(k1, ms);
          acc.off(k1 | (1u << ms), (ud * s) * s2, 0.0);
        }
        if (bit(m, o + ns) == 0 && bit(m, ms) == 1) {
          double s = jw_sign(m, ms);
          uint32_t k1 = m & ~(1u << ms);
          double s2 = jw_sign(k1, o + ns);
          acc.off(k1 | (1u << (o + ns)), (ud * s) * s2, 0.0);
        }
      }
  }
}

// -------------------------------------------------- symbolic row generator
// The off-diagonal terms of gen_row as state-independent candidates, in the
// same order: candidate c acts on a state m iff (m & req_mask) == req_val;
// its element is then (re, im) * sign at the row of m ^ flip, with the
// Jordan-Wigner sign of the operator string o_1 .. o_n (applied in that
// order, o_j at bit p_j):
//   sign = (-1)^( popc(m & smask) + c0 ),  smask = XOR_j (2^p_j - 1),
//   c0 = #{ i < j : p_i < p_j }  (each earlier flip below p_j changes the
//   parity that jw_sign(state_{j-1}, p_j) counts by one).
// (re, im) is gen_row's value before the signs (hr, -hi); multiplying by the
// +-1 factors in any grouping gives the same bits.  gen_row passes a literal
// 0.0 imaginary part for the two- and four-operator interaction terms (Jx,
// Jp, superc pairs, nonSU2 spin-flip hybridisation): im_signed = 0 keeps it
// unsigned there.  The matrix-free kernel
// (k_direct) evaluates these per lane instead of re-running gen_row's
// branchy loops; direct_candidates_check compares the two on sample states.
struct DirCand {
  uint32_t req_mask, req_val, flip, smask;
  int32_t c0, im_signed;
  double re, im;
};

struct CandBuilder {
  DirCand c{};
  uint32_t need1 = 0, need0 = 0;
  int pos[4];
  int nops = 0;
  bool ok = true;
  void req(int b, int v) {
    const uint32_t m = 1u << b;
    if (v) { ok = ok && !(need0 & m); need1 |= m; }
    else { ok = ok && !(need1 & m); need0 |= m; }
  }
  void op(int p) { pos[nops++] = p; }
  bool finish(double re, double im, bool im_signed = false) {
    if (!ok) return false;  // contradictory bit conditions: gen_row never fires
    c.req_mask = need1 | need0;
    c.req_val = need1;
    c.flip = 0;
    c.smask = 0;
    int c0 = 0;
    for (int j = 0; j < nops; j++) {
      c.flip ^= 1u << pos[j];
      c.smask ^= pos[j] == 0 ? 0u : ((1u << pos[j]) - 1u);
      for (int i = 0; i < j; i++) c0 += pos[i] < pos[j];
    }
    c.c0 = c0 & 1;
    c.im_signed = im_signed ? 1 : 0;
    c.re = re;
    c.im = im;
    return true;
  }
};

// Host: the candidates of gen_row (identical loop structure and conditions).
template <class Vec>
inline void direct_candidates(const EdModel& M, Vec& out) {
  const int ns = M.ns, norb = M.norb, nbath = M.nbath, S = M.S;
  auto hop = [&](int a, int b, double re, double im, bool signed_im = true) {  // c+_a c_b: bit b = 1, bit a = 0
    CandBuilder cb;
    cb.req(b, 1);
    cb.req(a, 0);
    cb.op(b);
    cb.op(a);
    if (cb.finish(re, im, signed_im)) out.push_back(cb.c);
  };
  // stored/Himp.f90:27-72
  for (int io = 0; io < norb; io++)
    for (int jo = 0; jo < norb; jo++) {
      double hr = M.hloc_re[0][0][io][jo], hi = M.hloc_im[0][0][io][jo];
      if (hr != 0.0 || hi != 0.0) hop(io, jo, hr, -hi);
      hr = M.hloc_re[S][S][io][jo];
      hi = M.hloc_im[S][S][io][jo];
      if (hr != 0.0 || hi != 0.0) hop(io + ns, jo + ns, hr, -hi);
    }
  // stored/Himp.f90:74-104
  if (M.mode == ED_MODE_NONSU2)
    for (int is = 0; is < 2; is++) {
      const int js = 1 - is;
      for (int io = 0; io < norb; io++)
        for (int jo = 0; jo < norb; jo++) {
          const double hr = M.hloc_re[is][js][io][jo], hi = M.hloc_im[is][js][io][jo];
          if (hr != 0.0 || hi != 0.0) hop(io + is * ns, jo + js * ns, hr, -hi);
        }
    }
  // stored/Hint.f90:60-123
  if (norb > 1 && M.jhflag) {
    for (int io = 0; io < norb; io++)
      for (int jo = 0; jo < norb; jo++) {
        if (io == jo) continue;
        CandBuilder cb;
        cb.req(jo, 1); cb.req(io + ns, 1); cb.req(jo + ns, 0); cb.req(io, 0);
        cb.op(jo); cb.op(io + ns); cb.op(jo + ns); cb.op(io);
        if (cb.finish(M.jx, 0.0)) out.push_back(cb.c);
      }
    for (int io = 0; io < norb; io++)
      for (int jo = 0; jo < norb; jo++) {
        if (io == jo) continue;
        CandBuilder cb;
        cb.req(jo, 1); cb.req(jo + ns, 1); cb.req(io + ns, 0); cb.req(io, 0);
        cb.op(jo); cb.op(jo + ns); cb.op(io + ns); cb.op(io);
        if (cb.finish(M.jp, 0.0)) out.push_back(cb.c);
      }
  }
  // stored/Hbath.f90:52-135
  if (M.bath == ED_BATH_REPLICA) {
    for (int k = 0; k < nbath; k++)
      for (int io = 0; io < norb; io++)
        for (int jo = 0; jo < norb; jo++)
          for (int sp = 0; sp < 2; sp++) {
            const int ss = sp == 0 ? 0 : S;
            const double hr = M.hb_re[ss][ss][io][jo][k], hi = M.hb_im[ss][ss][io][jo][k];
            if (hr != 0.0 || hi != 0.0) hop(M.stride[io][k] + sp * ns, M.stride[jo][k] + sp * ns, hr, -hi);
          }
    if (M.mode == ED_MODE_NONSU2)
      for (int k = 0; k < nbath; k++)
        for (int is = 0; is < 2; is++) {
          const int js = 1 - is;
          for (int io = 0; io < norb; io++)
            for (int jo = 0; jo < norb; jo++) {
              const double hr = M.hb_re[is][js][io][jo][k], hi = M.hb_im[is][js][io][jo][k];
              if (hr != 0.0 || hi != 0.0) hop(M.stride[io][k] + is * ns, M.stride[jo][k] + js * ns, hr, -hi);
            }
        }
  }
  // stored/Hbath.f90:142-178
  if (M.mode == ED_MODE_SUPERC)
    for (int o = 0; o < M.ne; o++)
      for (int k = 0; k < nbath; k++) {
        const int ms = M.stride[o][k];
        const double dd = M.d[0][o][k];
        if (dd == 0.0) continue;
        {
          CandBuilder cb;
          cb.req(ms, 1); cb.req(ms + ns, 1);
          cb.op(ms); cb.op(ms + ns);
          if (cb.finish(dd, 0.0)) out.push_back(cb.c);
        }
        {
          CandBuilder cb;
          cb.req(ms, 0); cb.req(ms + ns, 0);
          cb.op(ms + ns); cb.op(ms);
          if (cb.finish(dd, 0.0)) out.push_back(cb.c);
        }
      }
  // stored/Himp_bath.f90:10-67
  for (int o = 0; o < norb; o++)
    for (int k = 0; k < nbath; k++) {
      const int ms = M.stride[o][k];
      for (int sp = 0; sp < 2; sp++) {
        const int ss = sp == 0 ? 0 : S;
        const double hr = M.hyb_re[ss][o][k], hi = M.hyb_im[ss][o][k];
        if (hr == 0.0 && hi == 0.0) continue;
        const int a = o + sp * ns, b = ms + sp * ns;
        hop(b, a, hr, -hi);  // bit a = 1, bit b = 0: c+_b c_a
        hop(a, b, hr, -hi);  // bit a = 0, bit b = 1: c+_a c_b
      }
    }
  // stored/Himp_bath.f90:70-128 (no u /= 0 test)
  if (M.mode == ED_MODE_NONSU2 && M.bath != ED_BATH_REPLICA)
    for (int o = 0; o < norb; o++)
      for (int k = 0; k < nbath; k++) {
        const int ms = M.stride[o][k];
        const double uu = M.u[0][o][k], ud = M.u[S][o][k];
        hop(ms + ns, o, uu, 0.0, false);
        hop(o, ms + ns, uu, 0.0, false);
        hop(ms, o + ns, ud, 0.0, false);
        hop(o + ns, ms, ud, 0.0, false);
      }
}

// Evaluate candidate c on state m: true if it fires; target state, sign.
ED_HD bool cand_apply(const DirCand& c, uint32_t m, uint32_t* k, double* sg) {
  if ((m & c.req_mask) != c.req_val) return false;
  *k = m ^ c.flip;
  *sg = ((__builtin_popcount(m & c.smask) + c.c0) & 1) ? -1.0 : 1.0;
  return true;
}

}  // namespace edg
