"""Model configurations of the committed fixtures (shared by
tests/golden/make_golden.py, the GPU tests and bench.py; data only, no oracle)."""
from edgpu.params import make_config

SEED = 20251015
C2_KW = dict(Norb=1, Nbath=7)                                              # configs[1]/[2]
C4_KW = dict(Norb=2, Nbath=5, Uloc=(2.0, 2.0, 0.0), Ust=1.0, Jh=0.5)     # configs[3]
C5_KW = dict(Norb=1, Nbath=6, Nspin=2, ed_mode="nonsu2")                  # configs[4]


def c2_config(bath="random", seed=SEED):
    return make_config(bath=bath, seed=seed, **C2_KW)


def c4_config(bath="random"):
    return make_config(bath=bath, seed=SEED, **C4_KW)


def c5_config(bath="random"):
    return make_config(bath=bath, seed=SEED, **C5_KW)


# Adversarial degeneracy-probe sector (tests/golden/make_adversarial.py): the
# configs[3] model with orbital 2's bath set equal to orbital 1's ("equal bath
# pairs": the orbital swap is then a symmetry and every level of the (1,3)
# sector is an exact pair) and an orbital-symmetric impurity level `ed` tuned
# so that two pairs from different swap blocks lie a chosen distance apart.
ADV_SECTOR = (1, 3)


def adv_config(ed):
    cfg = make_config(bath="random", seed=SEED, **C4_KW)
    cfg.bath.e[:, 1, :] = cfg.bath.e[:, 0, :]
    cfg.bath.v[:, 1, :] = cfg.bath.v[:, 0, :]
    cfg.impHloc[0, 0, 0, 0] = ed
    cfg.impHloc[0, 0, 1, 1] = ed
    return cfg
