/* CPU ORACLE for hypre-ve_amd -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's BoomerAMG *solve* path
 * (SX-Aurora/hypre-ve, src/), used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker.  Nothing in the product
 * (hypre-ve_amd/, include/) links, loads or calls this code.
 *
 * Parity pin: the oracle's solve on the setup hierarchy reproduces the
 * reference's own saved outputs (src/test/TEST_ij/default.saved: average
 * convergence factor and grid/operator/cycle complexity), see
 * tests/test_oracle_golden.py.
 *
 * The reference C build is not used: it needs the configure-generated
 * HYPRE_config.h (src/config/HYPRE_config.h.in) and an MPI, neither of which
 * exists here, so it is treated as unbuildable ("Oracle").
 */
#ifndef HVE_ORACLE_H
#define HVE_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int nrows, ncols;
  const int *i, *j;
  const double *a;
} orc_csr;

#define ORC_MAX_LEVELS 40

typedef struct {
  int num_levels;
  orc_csr A[ORC_MAX_LEVELS];
  orc_csr P[ORC_MAX_LEVELS]; /* P[l]: n_l x n_{l+1}; unused on the coarsest level */
  const int *cf[ORC_MAX_LEVELS];
  const double *l1[ORC_MAX_LEVELS];
  int coarse_n;               /* dense coarsest operator for relax type 9 */
  const double *coarse_A;     /* row-major n x n, as hypre_GaussElimSetup builds it */
  int relax_type[4];          /* [0]: the user relax type (one-level smoother, -1 = 6) */
  int num_sweeps[4];
  double relax_weight, omega;
  int relax_order, cycle_type, num_blocks;
  orc_csr R[ORC_MAX_LEVELS]; /* optional P[l]^T with ascending rows (i == NULL: scatter) */
  /* Chebyshev smoother (relax type 16): per level 1/sqrt(a_ii) (scaled
   * variant) and the polynomial coefficients; order and scaling */
  const double *cheby_ds[ORC_MAX_LEVELS];
  double cheby_coefs[ORC_MAX_LEVELS][5];
  int cheby_order, cheby_scale;
  /* optional per-level hybrid-GS block starts (gs_nblocks[l] + 1 entries):
   * the blocks of an N-rank run; NULL = hypre's num_blocks thread partition */
  const int *gs_blocks[ORC_MAX_LEVELS];
  int gs_nblocks[ORC_MAX_LEVELS];
  /* optional per-level relax_weight / omega (par_cycle.c reads
   * relax_weight[level], omega[level]); used when lev_weights != 0 */
  int lev_weights;
  double lev_w[ORC_MAX_LEVELS], lev_omega[ORC_MAX_LEVELS];
} orc_amg;

/* OpenMP threads the row-parallel loops use (1 without OpenMP). */
int orc_num_threads(void);

/* seq_mv/csr_matvec.c:24 hypre_CSRMatrixMatvecOutOfPlaceHost:
 * y = alpha*A*x + beta*b (generic non-VE path, one thread). */
void orc_matvec(double alpha, const orc_csr *A, const double *x, double beta,
                const double *b, double *y);
/* seq_mv/csr_matvec.c:424 hypre_CSRMatrixMatvecTHost: y = alpha*A^T*x + beta*y */
void orc_matvecT(double alpha, const orc_csr *A, const double *x, double beta, double *y);

/* parcsr_ls/par_relax.c:31 hypre_BoomerAMGRelax (+ ams.c:41 for type 18) */
int orc_relax(const orc_csr *A, const double *f, const int *cf, int relax_type,
              int relax_points, double relax_weight, double omega, const double *l1,
              int num_blocks, double *u, double *vtemp, double *ztemp);

/* parcsr_ls/par_cheby.c:166 hypre_ParCSRRelax_Cheby_Solve (variant 0 and 1
 * share the solve; the coefficients differ). v, r: temporaries of n. */
int orc_cheby(const orc_csr *A, const double *f, const double *ds, const double *coefs, int order, int scale,
              double *u, double *v, double *r);

/* parcsr_ls/par_cycle.c:22 hypre_BoomerAMGCycle.  F[l], U[l] per level.
 * Returns cycle_op_count contribution via *op_count (may be NULL). */
int orc_cycle(const orc_amg *amg, double **F, double **U, double *op_count);

/* parcsr_ls/par_amg_solve.c:22 hypre_BoomerAMGSolve.
 * stats[0]=iterations, [1]=final rel. residual, [2]=avg conv factor,
 * [3]=cycle complexity (print-level accounting), [4]=initial residual norm. */
int orc_amg_solve(const orc_amg *amg, const double *f, double *u, double tol,
                  int min_iter, int max_iter, int converge_type, double *stats);

/* krylov/pcg.c:271 hypre_PCGSolve with BoomerAMG (1 V-cycle, tol 0) as
 * preconditioner (two_norm selectable).  stats[0]=iterations, [1]=rel. res. */
int orc_pcg_amg(const orc_amg *amg, const double *b, double *x, double tol,
                int max_iter, int two_norm, double *stats);

/* inner product in index order */
double orc_dot(int n, const double *x, const double *y);

#ifdef __cplusplus
}
#endif
#endif
