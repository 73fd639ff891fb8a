// ed_persist_launch.hip — the k_lanc_persist instantiations (one-workgroup
// persistent Lanczos, ed_persist.hpp) and their dispatch on the sector's
// register-layout geometry.  A translation unit of its own: these ~150
// instantiations are half of the library's device compile.
#include "ed_host.hpp"
#include "ed_kernels.hpp"
#include "ed_persist.hpp"

namespace edg {

template <bool HC, bool VC, int MODE, int RPT, int E = 1>
static int persist_launch_t(const PersistGeom& s, const PersistRun<HC>& run, int64_t lds, hipStream_t st, int nb) {
  if constexpr ((MODE == 2 || MODE == 3) && RPT * E > preg_cap(HC, VC)) {
    return fail(ED_ERR_UNSUPPORTED, "register-resident ELL exceeds the spill-free budget");
  } else if constexpr (MODE == 4 && (HC || (VC ? !pkr_fits_c512(E, RPT) : !pkr_fits(E, RPT)))) {
    return fail(ED_ERR_UNSUPPORTED, "Kronecker register layout: real H within the register budget");
  } else {
  constexpr int NT = MODE >= 2 ? kPRegBlock : kPBlock;
  auto fn = k_lanc_persist<HC, VC, MODE, RPT, E, NT>;
  HIPCK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(fn, dim3(nb), dim3(NT), (size_t)lds, st, run);
  HIPCK(hipGetLastError());
  return ED_OK;
  }
}

template <bool HC, bool VC, int MODE, int W>
static int persist_launch_e(const PersistGeom& s, const PersistRun<HC>& run, int64_t lds, hipStream_t st, int nb) {
  switch (MODE == 2 ? s.preg_rpt : MODE == 3 ? s.kreg_rpt : s.pkr_rpt) {
    case 2: return persist_launch_t<HC, VC, MODE, 2, W>(s, run, lds, st, nb);
    case 4: return persist_launch_t<HC, VC, MODE, 4, W>(s, run, lds, st, nb);
    case 6: return persist_launch_t<HC, VC, MODE, 6, W>(s, run, lds, st, nb);
    case 8: return persist_launch_t<HC, VC, MODE, 8, W>(s, run, lds, st, nb);
    default: return persist_launch_t<HC, VC, MODE, 10, W>(s, run, lds, st, nb);
  }
}

template <bool HC, bool VC, int MODE>
static int persist_launch_m(const PersistGeom& s, const PersistRun<HC>& run, int64_t lds, hipStream_t st, int nb = 1) {
  if constexpr (MODE == 4) {
    if constexpr (HC) {
      return fail(ED_ERR_UNSUPPORTED, "MODE 4 needs a real H");
    } else {
      return s.pkr_E == 4 ? persist_launch_e<HC, VC, 4, 4>(s, run, lds, st, nb)
                           : persist_launch_e<HC, VC, 4, 8>(s, run, lds, st, nb);
    }
  } else if constexpr (MODE >= 2) {
    switch (MODE == 2 ? s.preg_E : s.kreg_W) {
      case 8: return persist_launch_e<HC, VC, MODE, 8>(s, run, lds, st, nb);
      case 12: return persist_launch_e<HC, VC, MODE, 12>(s, run, lds, st, nb);
      case 14: return persist_launch_e<HC, VC, MODE, 14>(s, run, lds, st, nb);
      default: return persist_launch_e<HC, VC, MODE, 16>(s, run, lds, st, nb);
    }
  } else {
  switch (persist_rpt01(s.dim)) {
    case 1: return persist_launch_t<HC, VC, MODE, 1>(s, run, lds, st, nb);
    case 2: return persist_launch_t<HC, VC, MODE, 2>(s, run, lds, st, nb);
    case 3: return persist_launch_t<HC, VC, MODE, 3>(s, run, lds, st, nb);
    case 4: return persist_launch_t<HC, VC, MODE, 4>(s, run, lds, st, nb);
    case 5: return persist_launch_t<HC, VC, MODE, 5>(s, run, lds, st, nb);
    case 6: return persist_launch_t<HC, VC, MODE, 6>(s, run, lds, st, nb);
    case 8: return persist_launch_t<HC, VC, MODE, 8>(s, run, lds, st, nb);
    case 10: return persist_launch_t<HC, VC, MODE, 10>(s, run, lds, st, nb);
    case 12: return persist_launch_t<HC, VC, MODE, 12>(s, run, lds, st, nb);
    default: return persist_launch_t<HC, VC, MODE, 16>(s, run, lds, st, nb);
  }
  }
}

template <bool HC, bool VC>
static int persist_launch_hv(int mode, const PersistGeom& g, const void* run, int64_t lds, hipStream_t st, int nb) {
  const PersistRun<HC>& r = *(const PersistRun<HC>*)run;
  switch (mode) {
    case 0: return persist_launch_m<HC, VC, 0>(g, r, lds, st, nb);
    case 1: return persist_launch_m<HC, VC, 1>(g, r, lds, st, nb);
    case 2: return persist_launch_m<HC, VC, 2>(g, r, lds, st, nb);
    case 3: return persist_launch_m<HC, VC, 3>(g, r, lds, st, nb);
    default: return persist_launch_m<HC, VC, 4>(g, r, lds, st, nb);
  }
}

int persist_launch(bool hc, bool vc, int mode, const PersistGeom& g, const void* run, int64_t lds,
                   hipStream_t st, int nb) {
  if (hc) {
    if (!vc) return fail(ED_ERR_ARG, "complex H needs complex vectors");
    if (mode == 4) return fail(ED_ERR_UNSUPPORTED, "MODE 4 needs real H");
    return persist_launch_hv<true, true>(mode, g, run, lds, st, nb);
  }
  return vc ? persist_launch_hv<false, true>(mode, g, run, lds, st, nb)
            : persist_launch_hv<false, false>(mode, g, run, lds, st, nb);
}

}  // namespace edg
