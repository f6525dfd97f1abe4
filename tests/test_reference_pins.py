"""Host setup + oracle pinned to the reference's own saved outputs of np > 1
`ij` runs (tests/golden/ij_rank_fixtures.json, from src/test/TEST_ij/*.saved).

One process reproduces an N-rank reference run through
hypreve_BoomerAMGSetRankEmulation: every row in ParCSR order (own columns,
then the rest), per-rank PMIS random streams (par_indepset.c:25), per-rank
HMIS first passes (par_coarsen.c:874), CF_marker_offd semantics
(par_coarsen.c:2296/2348), ext+i truncation over [P_diag | P_offd]
(par_csr_matrix.c:2671), per-rank random vectors in the Chebyshev eigenvalue
estimate (par_relax_more.c:209) and one hybrid-GS block per rank
(par_relax.c with num_procs > 1).  The inputs are the -P process grid's
GenerateLaplacian[27pt] matrix and ij -rhsrand's per-rank random right-hand
side (tests/ij_emul.py).

This pins, against reference-held numbers: PMIS, PMIS1 and HMIS; ext+i with
Pmx 0 and 4; 7- and 27-point operators; relax 0 and 18 C/F-ordered, 18, the
l1 hybrid GS 13/14 (also C/F-ordered and weighted, w = 1.1), hybrid GS 4 up,
6 and 8 under PCG, Chebyshev (order 2/3, unscaled, variant 1),
BoomerAMG-PCG, and aggressive coarsening (HMIS second pass on S*S + 2S with
local measures per rank, multipass interpolation, 1 and 10 aggressive levels,
7- and 27-point: agg_interp.out.4/8, coarsening.out.7), and the extended /
extended+i interpolations in matrix-matrix form (interp.out.7/8), whose
hypre_ParMatmul products follow its np > 1 entry order (other-rank columns
first) under the emulation, and the 2-stage aggressive interpolations
agg_interp_type 5 / 7 with interp_type 18 (agg_interp.out.14/15/19).
agg_interp.out.20 (10 aggressive levels of type 7, agg_P12_mx 4) reaches the
saved 11 iterations but a final residual of 1.647026e-09 against 1.654514e-09:
test_agg_interp_out20_band keeps it as a band until that is found.
Round 5 adds the classical 2-stage interpolations agg_interp_type 1 (ext+i,
then partial ext+i, partial.c:16) and 3 (ext, then partial ext, partial.c:1855):
agg_interp.out.1/3/5/7/9 match every printed digit (1 and 10 aggressive
levels, agg_Pmx 4, agg_tr 0.3 / agg_P12_tr 0.2, agg_P12_mx 3).  Type 6 (MM
ext+i, then partial ext+i) reaches agg_interp.out.16's 9 iterations with
5.533979e-09 against 6.146679e-09 (test_agg_interp_out16_band).  The two open
cases share one thing no exact case has: agg_P12_mx truncating a first stage
built in matrix-matrix form (types 6 / 7), so the entry order that truncation's
tie-breaking sees there is the suspect.
The redundant coarse-grid AMG (seq_threshold, par_amg_setup.c:2880-2897,
gen_redcs_mat.c:18) reproduces solvers.out.105/106 (80^3 on 8 ranks, a
one-process BoomerAMG below 100 rows) to every printed digit;
test_seq_threshold_has_teeth shows the number moves without it.
Systems AMG, unknown approach (-sysL 3 -nf 3: par_laplace.c:394's
interleaved 3-function Laplacian, strength and weak lumping within a
function, par_strength.c:254 / par_lr_interp.c:1727 / par_multi_interp.c:1229,
coarse functions from the C points) reproduces agg_interp.out.10 (multipass,
10 aggressive levels), agg_interp.out.11 (2-stage ext+i) and
solvers.out.107/108 (with the redundant coarse grid) to every printed digit;
test_systems_amg_has_teeth shows num_functions 1 gives other numbers.
The Ruge first pass alone (coarsen_type 11, ij -ruge1p: par_coarsen.c:1347,
measure-0 points F) reproduces coarsening.out.9 (local measures per rank) and
coarsening.out.8 (-gm: global measures, other ranks' dependents counted,
par_coarsen.c:1088-1108);
default.out.0 (np 1, random PMIS) and solvers.out.sysu (-sysL 2 -nf 2, the
default solver) match every printed digit, and FCF-Jacobi (relax 17,
par_relax_more.c:661) smoother.out.14; ij -rotate's 2-D operator
(par_rotate_7pt.c, tests/ij_emul.py) under Chebyshev smoother.out.19, and
ij -vardifconv's jumping coefficients (par_vardifconv.c, its own right-hand
side, ij's random initial guess) with a 5-step CG eigenvalue estimate
smoother.out.20; the reference's own 2-rank elasticity matrix (TEST_ij/A.0000*,
kept as tests/golden/ij_elast_A.npz by scripts/make_file_fixtures.py) under
2-function systems AMG and PCG: elast.out.7.
Extended+i where no common C point (interp_type 7, par_lr_interp.c:1932)
matches interp.out.1/4 (Pmx 0 and 4) to every printed digit.
Standard interpolation (interp_type 8, par_lr_interp.c:22) matches
interp.out.2 (Pmx 0) in every printed digit; interp.out.5 (Pmx 4) has both
complexities exact and the convergence factor 0.203484 against 0.203482
(test_interp_out5_band).
"""
import json
import os

import numpy as np
import pytest
import scipy.sparse as sp

import ij_emul

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "ij_rank_fixtures.json")))["cases"]


def build(hv, case):
    prob = case["problem"]
    b_gen = None
    if prob.get("file"):  # a matrix the reference's tests read with ij -fromfile (scripts/make_file_fixtures.py)
        z = np.load(os.path.join(HERE, "golden", prob["file"]))
        n = len(z["indptr"]) - 1
        A_s = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(n, n))
        starts = [int(v) for v in z["starts"]]
    elif prob.get("rotate"):
        A_s, starts = ij_emul.rotate_ranks(*prob["n"], *prob["P"], *prob["rotate"])
    elif prob.get("vardifconv"):
        A_s, starts, b_gen = ij_emul.vardifconv_ranks(*prob["n"], *prob["P"], prob["vardifconv"])
    elif prob.get("sysL"):
        A_s, starts = ij_emul.sys_laplacian_ranks(*prob["n"], *prob["P"], nf=prob["sysL"])
    else:
        A_s, starts = ij_emul.laplacian_ranks(*prob["n"], *prob["P"], c=tuple(prob.get("c", (1.0, 1.0, 1.0))),
                                              pt27=prob["stencil"] == 27)
    A = hv.ParCSRMatrix.from_scipy(A_s)
    kw = hv.ij_amg_defaults(0 if case["solver"] == "amg" else 1)
    kw.update(num_blocks=1)
    st = dict(case["settings"])
    for key in ("cycle_relax_type", "cycle_num_sweeps"):
        if key in st:
            st[key] = {int(k): v for k, v in st[key].items()}
    kw.update(st)
    amg = hv.BoomerAMG(**kw)
    amg.set_rank_emulation(starts)
    if case["rhs"] == "generated":  # the generator's own right-hand side (ij build_rhs_type 6)
        b = b_gen
    elif case["rhs"] == "rhsrand":
        b = ij_emul.rhsrand(starts)
    elif case["rhs"] == "xisone":  # ij -xisone: b = A * ones (ij.c:629)
        b = A_s @ np.ones(A.n)
    else:
        b = np.ones(A.n)
    return A, amg, b, starts


def initial_guess(case, starts, n):
    """x0: zero, or ij's per-rank random guess (build_src_type 5)."""
    return ij_emul.rand_guess(starts) if case.get("x0") == "rand" else np.zeros(n)


def check_stats(case, amg, st=None, it=None, rr=None):
    exp = case["expect"]
    if "grid" in exp:
        g, o, _ = amg.complexities()
        assert f"{g:f}" == f"{exp['grid']:f}"
        assert f"{o:f}" == f"{exp['operator']:f}"
    if "conv_factor" in exp:
        assert f"{st['conv_factor']:f}" == f"{exp['conv_factor']:f}"
        assert abs(st["cycle_complexity"] - exp["cycle"]) < 1.5e-6
    if "iterations" in exp:
        assert it == exp["iterations"]
        assert f"{rr:e}" == f"{exp['rel_res']:e}"


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_rank_fixture(hv, orc, case):
    A, amg, b, starts = build(hv, case)
    amg.setup_host(A)
    O = orc.OracleAMG(amg)
    x = initial_guess(case, starts, A.n)
    if case["solver"] == "amg":
        st = O.solve(b, x, 1e-8, 100)
        check_stats(case, amg, st, st["iterations"], st["rel_res"])
    else:
        it, rr = O.pcg(b, x, 1e-8, 1000, 1)
        check_stats(case, amg, None, it, rr)
    amg.destroy()
    A.destroy()


def test_emulation_has_teeth(hv, orc):
    """Without the emulation (one process over the same matrix) coarsening.out.13
    and smoother.out.0 give other numbers: the pins depend on the per-rank
    behaviour, not just on the matrix."""
    for name in ("coarsening.out.13", "smoother.out.0"):
        case = next(c for c in CASES if c["name"] == name)
        A, amg, b, _ = build(hv, case)
        amg.set_rank_emulation(None)
        amg.setup_host(A)
        st = orc.OracleAMG(amg).solve(b, np.zeros(A.n), 1e-8, 100)
        exp = case["expect"]
        same = (st["iterations"] == exp.get("iterations") and f"{st['rel_res']:e}" == f"{exp.get('rel_res', 0):e}") \
            or f"{st['conv_factor']:f}" == f"{exp.get('conv_factor', -1):f}"
        assert not same, name


def test_rank_order_rows(hv):
    """Every level's rows are in ParCSR order under the emulation: the rank's own
    columns (diagonal first) before the other ranks' columns."""
    case = next(c for c in CASES if c["name"] == "interp.out.3")
    A, amg, b, starts = build(hv, case)
    amg.setup_host(A)
    rs = list(starts)
    for l in range(amg.num_levels()):
        ip, jj, vv, (nr, nc) = amg.level_matrix(l, 0)
        own = np.searchsorted(rs, np.arange(nr), side="right") - 1
        for i in range(nr):
            cols = jj[ip[i]:ip[i + 1]]
            if len(cols):
                assert cols[0] == i
            mine = own[np.clip(cols, 0, nr - 1)] == own[i]
            # own-rank entries form a prefix of the row
            k = int(np.argmin(mine)) if not mine.all() else len(mine)
            assert mine[:k].all() and not mine[k:].any()
        if l + 1 < amg.num_levels():
            cf = amg.level_vector(l, 0)
            pref = np.concatenate([[0], np.cumsum(cf == 1)])
            rs = [int(pref[s]) for s in rs]


def test_agg_interp_out20_band(hv, orc):
    """agg_interp.out.20 (mpirun -np 8 ./ij -rhsrand -n 30 29 31 -P 2 2 2
    -agg_nl 10 -agg_interp 7 -agg_Pmx 4 -agg_P12_mx 4 -solver 1 -rlx 6):
    saved 11 iterations, 1.654514e-09; not yet digit-exact (module docstring)."""
    base = next(c for c in CASES if c["name"] == "agg_interp.out.4")
    case = dict(base)
    case["settings"] = {"agg_num_levels": 10, "agg_interp_type": 7, "agg_P_max_elmts": 4, "agg_P12_max_elmts": 4,
                        "relax_type": 6}
    A, amg, b, _ = build(hv, case)
    amg.setup_host(A)
    it, rr = orc.OracleAMG(amg).pcg(b, np.zeros(A.n), 1e-8, 1000, 1)
    assert it == 11
    assert abs(rr - 1.654514e-09) < 0.01 * 1.654514e-09


def test_agg_interp_out16_band(hv, orc):
    """agg_interp.out.16 (mpirun -np 8 ./ij -rhsrand -n 30 29 31 -P 2 2 2
    -agg_nl 1 -agg_interp 6 -agg_Pmx 4 -agg_P12_mx 4 -solver 1 -rlx 6):
    saved 9 iterations, 6.146679e-09; not yet digit-exact (module docstring)."""
    base = next(c for c in CASES if c["name"] == "agg_interp.out.4")
    case = dict(base)
    case["settings"] = {"agg_num_levels": 1, "agg_interp_type": 6, "agg_P_max_elmts": 4, "agg_P12_max_elmts": 4,
                        "relax_type": 6}
    A, amg, b, _ = build(hv, case)
    amg.setup_host(A)
    it, rr = orc.OracleAMG(amg).pcg(b, np.zeros(A.n), 1e-8, 1000, 1)
    assert it == 9
    assert abs(rr - 6.146679e-09) < 0.15 * 6.146679e-09


def test_interp_out5_band(hv, orc):
    """interp.out.5 (mpirun -np 4 ./ij -rhsrand -n 15 15 10 -P 2 2 1
    -interptype 8): complexities to every printed digit, convergence factor
    within 1e-5 of the saved 0.203482 (module docstring)."""
    base = next(c for c in CASES if c["name"] == "interp.out.2")
    case = dict(base)
    case["settings"] = {"interp_type": 8}
    A, amg, b, _ = build(hv, case)
    amg.setup_host(A)
    g, o, _ = amg.complexities()
    assert f"{g:f}" == "1.582667" and f"{o:f}" == "2.662245"
    st = orc.OracleAMG(amg).solve(b, np.zeros(A.n), 1e-8, 100)
    assert abs(st["conv_factor"] - 0.203482) < 1e-5


def test_seq_threshold_has_teeth(hv, orc):
    """Without seq_threshold the same 8-rank run ends at 3.104551e-09, not the
    saved 3.104258e-09: the pin depends on the redundant coarse-grid AMG."""
    case = dict(next(c for c in CASES if c["name"] == "solvers.out.105"))
    case["settings"] = {k: v for k, v in case["settings"].items() if k != "seq_threshold"}
    A, amg, b, _ = build(hv, case)
    amg.setup_host(A)
    it, rr = orc.OracleAMG(amg).pcg(b, np.zeros(A.n), 1e-8, 1000, 1)
    assert f"{rr:e}" != "3.104258e-09"


def test_systems_amg_has_teeth(hv, orc):
    """agg_interp.out.10's system with num_functions 1 (strength across
    functions) ends elsewhere than the saved 22 iterations / 8.737365e-09."""
    case = dict(next(c for c in CASES if c["name"] == "agg_interp.out.10"))
    case["settings"] = {k: v for k, v in case["settings"].items() if k != "num_functions"}
    A, amg, b, _ = build(hv, case)
    amg.setup_host(A)
    it, rr = orc.OracleAMG(amg).pcg(b, np.zeros(A.n), 1e-8, 1000, 1)
    assert (it, f"{rr:e}") != (22, "8.737365e-09")


def test_global_measures_have_teeth(hv, orc):
    """coarsening.out.8 with local measures (measure_type 0) misses the saved
    13 iterations / 3.043813e-09: the other ranks' dependents matter."""
    case = dict(next(c for c in CASES if c["name"] == "coarsening.out.8"))
    case["settings"] = {"coarsen_type": 11, "measure_type": 0}
    A, amg, b, _ = build(hv, case)
    amg.setup_host(A)
    st = orc.OracleAMG(amg).solve(b, np.zeros(A.n), 1e-8, 100)
    assert (st["iterations"], f"{st['rel_res']:e}") != (13, "3.043813e-09")
