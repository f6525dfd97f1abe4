/* CPU ORACLE for hypre-ve_amd -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restates, statement for statement, the single-process (num_procs == 1)
 * branches of the reference's solve-phase routines.  Block-parallel
 * ("hybrid") smoothers take the reference's OpenMP thread partition as the
 * explicit parameter num_blocks (par_relax.c: size = n/num_threads, rest = ...).
 * Compiled with -ffp-contract=off so every a*b+c rounds twice, as the
 * reference's generic C path does on a host without FMA contraction.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

double orc_dot(int n, const double *x, const double *y) {
  double s = 0.0;
  for (int i = 0; i < n; i++) s += x[i] * y[i];
  return s;
}

#ifdef _OPENMP
#include <omp.h>
#endif
int orc_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ---- seq_mv/csr_matvec.c:24-330 (generic, non-rownnz path) ---- */
void orc_matvec(double alpha, const orc_csr *A, const double *x, double beta,
                const double *b, double *y) {
  const int n = A->nrows;
  const int *Ai = A->i, *Aj = A->j;
  const double *Aa = A->a;
  double *xcopy = NULL;
  if (alpha == 0.0) {
#pragma omp parallel for schedule(static) if (n > 8192)
    for (int i = 0; i < n; i++) y[i] = beta * b[i];
    return;
  }
  if (x == y) {
    xcopy = (double *)malloc(sizeof(double) * (size_t)A->ncols);
    memcpy(xcopy, x, sizeof(double) * (size_t)A->ncols);
    x = xcopy;
  }
  const double temp = beta / alpha;
  /* rows are independent: the OpenMP split changes no row's arithmetic */
#pragma omp parallel for schedule(static) if (n > 8192)
  for (int i = 0; i < n; i++) {
    double t;
    if (temp == 0.0) {
      t = 0.0;
      if (alpha == -1.0) { for (int k = Ai[i]; k < Ai[i + 1]; k++) t -= Aa[k] * x[Aj[k]]; y[i] = t; }
      else { for (int k = Ai[i]; k < Ai[i + 1]; k++) t += Aa[k] * x[Aj[k]]; y[i] = (alpha == 1.0) ? t : alpha * t; }
    } else if (temp == -1.0) {
      if (alpha == 1.0) { t = -b[i]; for (int k = Ai[i]; k < Ai[i + 1]; k++) t += Aa[k] * x[Aj[k]]; y[i] = t; }
      else if (alpha == -1.0) { t = b[i]; for (int k = Ai[i]; k < Ai[i + 1]; k++) t -= Aa[k] * x[Aj[k]]; y[i] = t; }
      else { t = -b[i]; for (int k = Ai[i]; k < Ai[i + 1]; k++) t += Aa[k] * x[Aj[k]]; y[i] = alpha * t; }
    } else if (temp == 1.0) {
      if (alpha == 1.0) { t = b[i]; for (int k = Ai[i]; k < Ai[i + 1]; k++) t += Aa[k] * x[Aj[k]]; y[i] = t; }
      else if (alpha == -1.0) { t = -b[i]; for (int k = Ai[i]; k < Ai[i + 1]; k++) t -= Aa[k] * x[Aj[k]]; y[i] = t; }
      else { t = b[i]; for (int k = Ai[i]; k < Ai[i + 1]; k++) t += Aa[k] * x[Aj[k]]; y[i] = alpha * t; }
    } else {
      if (alpha == 1.0) { t = b[i] * temp; for (int k = Ai[i]; k < Ai[i + 1]; k++) t += Aa[k] * x[Aj[k]]; y[i] = t; }
      else if (alpha == -1.0) { t = -b[i] * temp; for (int k = Ai[i]; k < Ai[i + 1]; k++) t -= Aa[k] * x[Aj[k]]; y[i] = t; }
      else { t = b[i] * temp; for (int k = Ai[i]; k < Ai[i + 1]; k++) t += Aa[k] * x[Aj[k]]; y[i] = alpha * t; }
    }
  }
  free(xcopy);
}

/* ---- seq_mv/csr_matvec.c:424 (one thread) ---- */
void orc_matvecT(double alpha, const orc_csr *A, const double *x, double beta, double *y) {
  const int nc = A->ncols;
  if (alpha == 0.0) { for (int i = 0; i < nc; i++) y[i] *= beta; return; }
  const double temp = beta / alpha;
  if (temp != 1.0) {
    if (temp == 0.0) for (int i = 0; i < nc; i++) y[i] = 0.0;
    else for (int i = 0; i < nc; i++) y[i] *= temp;
  }
  for (int i = 0; i < A->nrows; i++)
    for (int k = A->i[i]; k < A->i[i + 1]; k++) y[A->j[k]] += A->a[k] * x[i];
  if (alpha != 1.0) for (int i = 0; i < nc; i++) y[i] *= alpha;
}

static void block_range(int n, int nb, int k, int *ns, int *ne) {
  int size = n / nb, rest = n - size * nb;
  if (k < rest) { *ns = k * size + k; *ne = (k + 1) * size + k + 1; }
  else { *ns = k * size + rest; *ne = (k + 1) * size + rest; }
}

/* hybrid GS (3 fwd, 4 bwd, 6 sym) and l1 hybrid GS (13, 14, 8).
 * par_relax.c:354 (3), :1875 (4), :2266 (6), :3492 (8), :4340 (13), :4732 (14).
 * Blocks: hypre's thread partition of num_blocks (block_range), or explicit
 * starts bst[0..nb] (the blocks an N-rank run sweeps: every rank's rows split
 * into its threads; off-rank columns read Vext, the pre-sweep values, as
 * off-block columns read tmp).
 * Weights 1 (par_relax.c:1040, :4387): res = f - sum a u (the diagonal
 * included for the l1 forms), u += res/l1 or u = res/a_ii.
 * Weighted (relax_weight or omega != 1, par_relax.c:1277, :3150, :3785, :4544):
 * Vtemp = tmp = u before the sweep; the diagonal entry skipped; in-block
 * res0 -= a u, res2 += a Vtemp; off-block res -= a tmp;
 * u *= 1 - w*omega; u += w*(omega*res + res0 + (1-omega)*res2) / d,
 * d = a_ii or l1_i.  A symmetric sweep keeps the one Vtemp for both halves. */
static void hybrid_gs(const orc_csr *A, const double *f, const int *cf, int relax_points,
                      const double *l1, int nb, const int *bst, int fwd, int bwd, int use_l1,
                      double w, double omega, double *u, double *tmp) {
  const int n = A->nrows;
  const int *Ai = A->i, *Aj = A->j;
  const double *Aa = A->a;
  const int weighted = (w != 1.0 || omega != 1.0);
  const double prod = 1.0 - w * omega, omo = 1.0 - omega;
  if (nb < 1) nb = 1;
  if (nb > 1 || weighted) memcpy(tmp, u, sizeof(double) * (size_t)n);
  /* blocks interact only through tmp: independent, as hypre's threads are */
#pragma omp parallel for schedule(dynamic, 1) if (nb > 1)
  for (int b = 0; b < nb; b++) {
    int ns, ne;
    if (bst) { ns = bst[b]; ne = bst[b + 1]; }
    else if (nb == 1) { ns = 0; ne = n; }
    else block_range(n, nb, b, &ns, &ne);
    for (int pass = 0; pass < 2; pass++) {
      if ((pass == 0 && !fwd) || (pass == 1 && !bwd)) continue;
      for (int q = 0; q < ne - ns; q++) {
        const int i = pass == 0 ? ns + q : ne - 1 - q;
        if (relax_points != 0 && cf[i] != relax_points) continue;
        if (weighted) {
          const double d = use_l1 ? l1[i] : Aa[Ai[i]];
          if (d == 0.0) continue;
          double res = f[i], res0 = 0.0, res2 = 0.0;
          for (int k = Ai[i] + 1; k < Ai[i + 1]; k++) {
            const int c = Aj[k];
            if (c >= ns && c < ne) {
              res0 -= Aa[k] * u[c];
              res2 += Aa[k] * tmp[c];
            } else {
              res -= Aa[k] * tmp[c];
            }
          }
          u[i] *= prod;
          u[i] += w * (omega * res + res0 + omo * res2) / d;
        } else if (use_l1) {
          if (l1[i] == 0.0) continue;
          double res = f[i];
          for (int k = Ai[i]; k < Ai[i + 1]; k++) {
            const int c = Aj[k];
            if (nb == 1 || (c >= ns && c < ne)) res -= Aa[k] * u[c];
            else res -= Aa[k] * tmp[c];
          }
          u[i] += res / l1[i];
        } else {
          const double d = Aa[Ai[i]];
          if (d == 0.0) continue;
          double res = f[i];
          for (int k = Ai[i] + 1; k < Ai[i + 1]; k++) {
            const int c = Aj[k];
            if (nb == 1 || (c >= ns && c < ne)) res -= Aa[k] * u[c];
            else res -= Aa[k] * tmp[c];
          }
          u[i] = res / d;
        }
      }
    }
  }
}

static int relax_impl(const orc_csr *A, const double *f, const int *cf, int relax_type,
                      int relax_points, double relax_weight, double omega, const double *l1,
                      int num_blocks, const int *bst, double *u, double *vtemp, double *ztemp);

int orc_relax(const orc_csr *A, const double *f, const int *cf, int relax_type,
              int relax_points, double relax_weight, double omega, const double *l1,
              int num_blocks, double *u, double *vtemp, double *ztemp) {
  return relax_impl(A, f, cf, relax_type, relax_points, relax_weight, omega, l1, num_blocks, NULL, u,
                    vtemp, ztemp);
}

static int relax_impl(const orc_csr *A, const double *f, const int *cf, int relax_type,
                      int relax_points, double relax_weight, double omega, const double *l1,
                      int num_blocks, const int *bst, double *u, double *vtemp, double *ztemp) {
  const int n = A->nrows;
  const int *Ai = A->i, *Aj = A->j;
  const double *Aa = A->a;
  switch (relax_type) {
    case 0: { /* par_relax.c:139 weighted Jacobi */
      const double omw = 1.0 - relax_weight;
      memcpy(vtemp, u, sizeof(double) * (size_t)n);
#pragma omp parallel for schedule(static) if (n > 8192)
      for (int i = 0; i < n; i++) {
        if (relax_points != 0 && cf[i] != relax_points) continue;
        const double d = Aa[Ai[i]];
        if (d == 0.0) continue;
        double res = f[i];
        for (int k = Ai[i] + 1; k < Ai[i + 1]; k++) res -= Aa[k] * vtemp[Aj[k]];
        u[i] *= omw;
        u[i] += relax_weight * res / d;
      }
      return 0;
    }
    case 18:
      if (relax_points != 0) {
        /* par_relax_more.c:991 hypre_ParCSRRelax_L1_Jacobi (par_cycle.c:398-415,
         * relax_order 1): Vtemp = u; rows of the class relax_points with a
         * nonzero diagonal: res = f - sum_j a_ij Vtemp_j (stored order, the
         * diagonal included), u_i += (w*res)/l1_i.  An empty row is skipped
         * (the reference would read the next row's first entry). */
        memcpy(vtemp, u, sizeof(double) * (size_t)n);
#pragma omp parallel for schedule(static) if (n > 8192)
        for (int i = 0; i < n; i++) {
          if (cf[i] != relax_points || Ai[i] == Ai[i + 1] || Aa[Ai[i]] == 0.0) continue;
          double res = f[i];
          for (int k = Ai[i]; k < Ai[i + 1]; k++) res -= Aa[k] * vtemp[Aj[k]];
          u[i] += (relax_weight * res) / l1[i];
        }
        return 0;
      }
      /* fall through: ams.c:41 hypre_ParCSRRelax type 1 (l1-scaled Jacobi) */
    case 7: { /* par_relax.c:3463 Jacobi through the matvec (l1 = diag); relax_points
               * is ignored (a C/F-ordered call runs a full sweep) */
      memcpy(vtemp, f, sizeof(double) * (size_t)n);
      orc_matvec(-relax_weight, A, u, relax_weight, vtemp, vtemp);
#pragma omp parallel for schedule(static) if (n > 8192)
      for (int i = 0; i < n; i++) u[i] += vtemp[i] / l1[i];
      return 0;
    }
    case 3: case 4: case 6: case 8: case 13: case 14: {
      const int fwd = (relax_type == 3 || relax_type == 6 || relax_type == 8 || relax_type == 13);
      const int bwd = (relax_type == 4 || relax_type == 6 || relax_type == 8 || relax_type == 14);
      const int use_l1 = (relax_type == 8 || relax_type == 13 || relax_type == 14);
      hybrid_gs(A, f, cf, relax_points, l1, num_blocks, bst, fwd, bwd, use_l1, relax_weight, omega, u,
                ztemp);
      return 0;
    }
    default:
      return 3;
  }
}

/* hypre_gselim (sstruct_ls/gselim.h) on a copy of the dense coarsest matrix,
 * as hypre_GaussElimSolve (par_gauss_elim.c:202) does for relax type 9. */
static void gauss_elim_solve(int n, const double *Amat, const double *f, double *u) {
  double *A = (double *)malloc(sizeof(double) * (size_t)n * n);
  double *x = (double *)malloc(sizeof(double) * (size_t)n);
  memcpy(A, Amat, sizeof(double) * (size_t)n * n);
  memcpy(x, f, sizeof(double) * (size_t)n);
  if (n == 1) {
    if (A[0] != 0.0) x[0] = x[0] / A[0];
  } else {
    for (int k = 0; k < n - 1; k++) {
      if (A[k * n + k] != 0.0) {
        double divA = 1.0 / A[k * n + k];
        for (int j = k + 1; j < n; j++) {
          if (A[j * n + k] != 0.0) {
            double factor = A[j * n + k] * divA;
            for (int m = k + 1; m < n; m++) A[j * n + m] -= factor * A[k * n + m];
            x[j] -= factor * x[k];
          }
        }
      }
    }
    for (int k = n - 1; k > 0; --k) {
      if (A[k * n + k] != 0.0) {
        x[k] /= A[k * n + k];
        for (int j = 0; j < k; j++)
          if (A[j * n + k] != 0.0) x[j] -= x[k] * A[j * n + k];
      }
    }
    if (A[0] != 0.0) x[0] /= A[0];
  }
  memcpy(u, x, sizeof(double) * (size_t)n);
  free(A);
  free(x);
}

/* ---- parcsr_ls/par_cycle.c:22 hypre_BoomerAMGCycle (smooth_num_levels = 0,
 * no grid_relax_points, no block mode) ---- */
int orc_cheby(const orc_csr *A, const double *f, const double *ds, const double *coefs, int order, int scale,
              double *u, double *v, double *r) {
  const int n = A->nrows;
  if (order > 4) order = 4;
  if (order < 1) order = 1;
  const int cheby_order = order - 1;
  double *orig_u = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
  if (!scale) {
    /* r = f - A u */
    orc_matvec(-1.0, A, u, 1.0, f, r);
    for (int i = 0; i < n; i++) {
      orig_u[i] = u[i];
      u[i] = r[i] * coefs[cheby_order];
    }
    for (int i = cheby_order - 1; i >= 0; i--) {
      orc_matvec(1.0, A, u, 0.0, NULL, v);
      const double mult = coefs[i];
      for (int j = 0; j < n; j++) u[j] = mult * r[j] + v[j];
    }
    for (int i = 0; i < n; i++) u[i] = orig_u[i] + u[i];
  } else {
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    /* tmp = -A u; r = D^{-1/2} (f + tmp) */
    orc_matvec(-1.0, A, u, 0.0, NULL, tmp);
    for (int j = 0; j < n; j++) r[j] = ds[j] * (f[j] + tmp[j]);
    for (int j = 0; j < n; j++) {
      orig_u[j] = u[j];
      u[j] = r[j] * coefs[cheby_order];
    }
    for (int i = cheby_order - 1; i >= 0; i--) {
      for (int j = 0; j < n; j++) tmp[j] = ds[j] * u[j];
      orc_matvec(1.0, A, tmp, 0.0, NULL, v);
      const double mult = coefs[i];
      for (int j = 0; j < n; j++) u[j] = mult * r[j] + ds[j] * v[j];
    }
    for (int j = 0; j < n; j++) u[j] = orig_u[j] + ds[j] * u[j];
    free(tmp);
  }
  free(orig_u);
  return 0;
}

int orc_cycle(const orc_amg *amg, double **F, double **U, double *op_count) {
  const int nl = amg->num_levels;
  int lev_counter[ORC_MAX_LEVELS];
  int nmax = 0;
  for (int l = 0; l < nl; l++) if (amg->A[l].nrows > nmax) nmax = amg->A[l].nrows;
  double *vtemp = (double *)calloc((size_t)nmax, sizeof(double));
  double *ztemp = (double *)calloc((size_t)nmax, sizeof(double));
  double ops = op_count ? *op_count : 0.0;
  int err = 0;
  lev_counter[0] = 1;
  for (int k = 1; k < nl; k++) lev_counter[k] = amg->cycle_type;
  int level = 0, cycle_param = 1, not_finished = 1;
  /* the level's hybrid-GS blocks: explicit (N-rank emulation) or num_blocks */
#define RELAX(pts)                                                                              \
  relax_impl(&amg->A[level], F[level], amg->cf[level], relax_type, (pts),                      \
             amg->lev_weights ? amg->lev_w[level] : amg->relax_weight,                          \
             amg->lev_weights ? amg->lev_omega[level] : amg->omega, amg->l1[level], amg->gs_blocks[level] ? amg->gs_nblocks[level] : amg->num_blocks, \
             amg->gs_blocks[level], U[level], vtemp, ztemp)
  while (not_finished) {
    int num_sweep, relax_type;
    if (nl > 1) {
      num_sweep = amg->num_sweeps[cycle_param];
      relax_type = amg->relax_type[cycle_param];
    } else {
      num_sweep = 1;
      relax_type = amg->relax_type[0] >= 0 ? amg->relax_type[0] : 6;
    }
    for (int j = 0; j < num_sweep; j++) {
      ops += (double)amg->A[level].i[amg->A[level].nrows];
      if (relax_type == 9 || relax_type == 99 || relax_type == 199) {
        gauss_elim_solve(amg->coarse_n, amg->coarse_A, F[level], U[level]);
      } else if (relax_type == 16) {
        /* par_cycle.c:445 scaled Chebyshev: Aux_F, Aux_U, Vtemp, Ztemp */
        err = orc_cheby(&amg->A[level], F[level], amg->cheby_ds[level], amg->cheby_coefs[level],
                        amg->cheby_order, amg->cheby_scale, U[level], vtemp, ztemp);
      } else if (relax_type == 17) {
        /* par_cycle.c:451 / par_relax_more.c:661 FCF-Jacobi: weighted Jacobi
         * (relax 0) over the F, then C, then F points, whatever relax_order;
         * one plain sweep on the coarsest level */
        const int pts[3] = {-1, 1, -1};
        relax_type = 0;
        if (level == nl - 1) err = RELAX(0);
        for (int q = 0; q < 3 && level != nl - 1 && !err; q++) err = RELAX(pts[q]);
        relax_type = 17;
      } else if (relax_type == 18 && !(amg->relax_order == 1 && cycle_param < 3)) {
        err = RELAX(0);
      } else {
        /* relax 18 with relax_order 1 (par_cycle.c:398-415): C/F-ordered
         * hypre_ParCSRRelax_L1_Jacobi twice; every other type through
         * hypre_BoomerAMGRelaxIF (par_relax_interface.c:19), which for relax 7
         * means two full sweeps (par_relax.c:3463 ignores relax_points) */
        if (amg->relax_order == 1 && cycle_param < 3) {
          int pts[2];
          if (cycle_param < 2) { pts[0] = 1; pts[1] = -1; } else { pts[0] = -1; pts[1] = 1; }
          for (int q = 0; q < 2 && !err; q++)
            err = RELAX(pts[q]);
        } else {
          err = RELAX(0);
        }
      }
      if (err) goto done;
    }
    --lev_counter[level];
    if (lev_counter[level] >= 0 && level != nl - 1) {
      const int fine = level, coarse = level + 1;
      memset(U[coarse], 0, sizeof(double) * (size_t)amg->A[coarse].nrows);
      orc_matvec(-1.0, &amg->A[fine], U[fine], 1.0, F[fine], vtemp);
      if (amg->R[fine].i) {
        /* hypre_CSRMatrixMatvecT (alpha 1, beta 0) scatters y[j] += a_ij x_i
         * for i ascending; R = P^T with ascending rows gathers the same terms
         * in the same order, so each F_c entry is bitwise the scatter's */
        const orc_csr *R = &amg->R[fine];
        double *Fc = F[coarse];
#pragma omp parallel for schedule(static) if (R->nrows > 8192)
        for (int j = 0; j < R->nrows; j++) {
          double t = 0.0;
          for (int k = R->i[j]; k < R->i[j + 1]; k++) t += R->a[k] * vtemp[R->j[k]];
          Fc[j] = t;
        }
      } else {
        orc_matvecT(1.0, &amg->P[fine], vtemp, 0.0, F[coarse]);
      }
      ++level;
      lev_counter[level] = lev_counter[level] > amg->cycle_type ? lev_counter[level] : amg->cycle_type;
      cycle_param = (level == nl - 1) ? 3 : 1;
    } else if (level != 0) {
      const int fine = level - 1, coarse = level;
      orc_matvec(1.0, &amg->P[fine], U[coarse], 1.0, U[fine], U[fine]);
      --level;
      cycle_param = 2;
    } else {
      not_finished = 0;
    }
  }
done:
  free(vtemp);
  free(ztemp);
  if (op_count) *op_count = ops;
  return err;
#undef RELAX
}

/* ---- parcsr_ls/par_amg_solve.c:22 ---- */
int orc_amg_solve(const orc_amg *amg, const double *f, double *u, double tol,
                  int min_iter, int max_iter, int converge_type, double *stats) {
  const int nl = amg->num_levels;
  const int n = amg->A[0].nrows;
  double *F[ORC_MAX_LEVELS], *U[ORC_MAX_LEVELS];
  F[0] = (double *)f;
  U[0] = u;
  for (int l = 1; l < nl; l++) {
    F[l] = (double *)calloc((size_t)amg->A[l].nrows, sizeof(double));
    U[l] = (double *)calloc((size_t)amg->A[l].nrows, sizeof(double));
  }
  double *vtemp = (double *)malloc(sizeof(double) * (size_t)n);
  double resid_nrm = 1.0, resid_nrm_init = 0.0, rhs_norm = 0.0, relative_resid = 1.0;
  double op_count = 0.0;
  int cycle_count = 0, err = 0;
  if (tol > 0.) {
    memcpy(vtemp, f, sizeof(double) * (size_t)n);
    orc_matvec(1.0, &amg->A[0], u, -1.0, vtemp, vtemp);
    resid_nrm = sqrt(orc_dot(n, vtemp, vtemp));
    resid_nrm_init = resid_nrm;
    if (converge_type == 0) {
      rhs_norm = sqrt(orc_dot(n, f, f));
      relative_resid = rhs_norm ? resid_nrm_init / rhs_norm : resid_nrm_init;
    } else {
      relative_resid = 1.0;
    }
  }
  while ((relative_resid >= tol || cycle_count < min_iter) && cycle_count < max_iter) {
    op_count = 0.0;
    err = orc_cycle(amg, F, U, &op_count);
    if (err) break;
    if (tol > 0.) {
      double old_resid = resid_nrm;
      (void)old_resid;
      orc_matvec(-1.0, &amg->A[0], u, 1.0, f, vtemp);
      resid_nrm = sqrt(orc_dot(n, vtemp, vtemp));
      if (converge_type == 0) relative_resid = rhs_norm ? resid_nrm / rhs_norm : resid_nrm;
      else relative_resid = resid_nrm / resid_nrm_init;
    }
    ++cycle_count;
  }
  double conv_factor = 1.0;
  if (cycle_count > 0 && resid_nrm_init) conv_factor = pow(resid_nrm / resid_nrm_init, 1.0 / (double)cycle_count);
  if (stats) {
    stats[0] = cycle_count;
    stats[1] = relative_resid;
    stats[2] = conv_factor;
    stats[3] = op_count / (double)amg->A[0].i[n];
    stats[4] = resid_nrm_init;
  }
  for (int l = 1; l < nl; l++) { free(F[l]); free(U[l]); }
  free(vtemp);
  return err;
}

/* ---- krylov/pcg.c:271 hypre_PCGSolve (stop_crit 0, rel_change 0, no
 * recompute, cf_tol 0) with BoomerAMG preconditioning: HYPRE_BoomerAMGSolve
 * with tol 0 and max_iter 1 performs exactly one cycle on a cleared vector. ---- */
int orc_pcg_amg(const orc_amg *amg, const double *b, double *x, double tol,
                int max_iter, int two_norm, double *stats) {
  const int n = amg->A[0].nrows;
  const orc_csr *A = &amg->A[0];
  double *r = (double *)malloc(sizeof(double) * (size_t)n);
  double *p = (double *)malloc(sizeof(double) * (size_t)n);
  double *s = (double *)malloc(sizeof(double) * (size_t)n);
  double bi_prod, eps, gamma, gamma_old, alpha, beta, sdotp;
  double i_prod = 0.0, i_prod_0 = 0.0;
  int i = 0, err = 0;
  double *F[ORC_MAX_LEVELS], *U[ORC_MAX_LEVELS];
  for (int l = 1; l < amg->num_levels; l++) {
    F[l] = (double *)calloc((size_t)amg->A[l].nrows, sizeof(double));
    U[l] = (double *)calloc((size_t)amg->A[l].nrows, sizeof(double));
  }
#define PRECOND(rr, zz)                                    \
  do {                                                     \
    memset((zz), 0, sizeof(double) * (size_t)n);           \
    F[0] = (double *)(rr); U[0] = (zz);                    \
    if (orc_cycle(amg, F, U, NULL)) { err = 4; goto done; } \
  } while (0)

  if (two_norm) {
    bi_prod = orc_dot(n, b, b);
  } else {
    PRECOND(b, p);
    bi_prod = orc_dot(n, p, b);
  }
  eps = tol * tol;
  if (!(bi_prod > 0.0)) {
    memcpy(x, b, sizeof(double) * (size_t)n);
    if (stats) { stats[0] = 0; stats[1] = 0; }
    goto done;
  }
  memcpy(r, b, sizeof(double) * (size_t)n);
  orc_matvec(-1.0, A, x, 1.0, r, r);
  PRECOND(r, p);
  gamma = orc_dot(n, r, p);
  i_prod_0 = two_norm ? orc_dot(n, r, r) : gamma;
  while ((i + 1) <= max_iter) {
    i++;
    orc_matvec(1.0, A, p, 0.0, s, s);
    sdotp = orc_dot(n, s, p);
    if (sdotp == 0.0) { if (i == 1) i_prod = i_prod_0; break; }
    alpha = gamma / sdotp;
    if (!(alpha > DBL_MIN)) { if (i == 1) i_prod = i_prod_0; break; }
    gamma_old = gamma;
    for (int q = 0; q < n; q++) x[q] += alpha * p[q];
    for (int q = 0; q < n; q++) r[q] += -alpha * s[q];
    PRECOND(r, s);
    gamma = orc_dot(n, r, s);
    i_prod = two_norm ? orc_dot(n, r, r) : gamma;
    if (i_prod / bi_prod < eps) break;
    if (!(gamma > DBL_MIN)) break;
    beta = gamma / gamma_old;
    for (int q = 0; q < n; q++) p[q] *= beta;
    for (int q = 0; q < n; q++) p[q] += 1.0 * s[q];
  }
  if (stats) {
    stats[0] = i;
    stats[1] = sqrt(i_prod / bi_prod);
  }
#undef PRECOND
done:
  for (int l = 1; l < amg->num_levels; l++) { free(F[l]); free(U[l]); }
  free(r); free(p); free(s);
  return err;
}
