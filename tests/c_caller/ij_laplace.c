/* A plain C caller of include/hypreve.h, written the way test/ij.c drives
 * hypre: the 3-D 7-point Laplacian assembled row by row through the IJ
 * interface (the entry order of par_laplace.c GenerateLaplacian: diagonal,
 * then z-, y-, x-, x+, y+, z+), b = A * 1 (ij -xisone), x = 0, then
 *   - BoomerAMG:  -pmis -Pmx 0 -rlx 0  (test/TEST_ij default.out.0 at 10^3)
 *   - PCG + BoomerAMG preconditioner (ij -solver 1: HMIS, ext+i Pmx 4, hybrid GS)
 * Prints "amg <iterations> <final rel. residual>" and "pcg <iterations> <res>".
 * Usage: ij_laplace [n]   (n^3 grid, default 10). */
#include <stdio.h>
#include <stdlib.h>

#include "hypreve.h"

#define CHECK(call)                                                            \
  do {                                                                         \
    HYPRE_Int rc_ = (call);                                                    \
    if (rc_ && rc_ != HYPRE_ERROR_CONV) {                                      \
      fprintf(stderr, "%s failed: %d (%s)\n", #call, (int)rc_, hypreve_LastErrorMessage()); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 10;
  const int N = n * n * n;
  HYPRE_IJMatrix ij;
  HYPRE_ParCSRMatrix A;
  HYPRE_IJVector ib, ix;
  HYPRE_ParVector b, x, one;
  HYPRE_Int i, its;
  HYPRE_Real res;

  CHECK(HYPRE_Init());
  CHECK(HYPRE_IJMatrixCreate(HYPRE_COMM_SELF, 0, N - 1, 0, N - 1, &ij));
  CHECK(HYPRE_IJMatrixSetObjectType(ij, HYPRE_PARCSR));
  CHECK(HYPRE_IJMatrixInitialize(ij));
  for (i = 0; i < N; i++) {
    const int ix_ = i % n, iy = (i / n) % n, iz = i / (n * n);
    HYPRE_BigInt row = i, cols[7];
    HYPRE_Complex vals[7];
    HYPRE_Int nc = 0;
    cols[nc] = i; vals[nc++] = 6.0;
    if (iz > 0) { cols[nc] = i - n * n; vals[nc++] = -1.0; }
    if (iy > 0) { cols[nc] = i - n; vals[nc++] = -1.0; }
    if (ix_ > 0) { cols[nc] = i - 1; vals[nc++] = -1.0; }
    if (ix_ + 1 < n) { cols[nc] = i + 1; vals[nc++] = -1.0; }
    if (iy + 1 < n) { cols[nc] = i + n; vals[nc++] = -1.0; }
    if (iz + 1 < n) { cols[nc] = i + n * n; vals[nc++] = -1.0; }
    CHECK(HYPRE_IJMatrixSetValues(ij, 1, &nc, &row, cols, vals));
  }
  CHECK(HYPRE_IJMatrixAssemble(ij));
  CHECK(HYPRE_IJMatrixGetObject(ij, (void **)&A));

  {
    HYPRE_BigInt part[2] = {0, N};
    CHECK(HYPRE_ParVectorCreate(HYPRE_COMM_SELF, N, part, &one));
    CHECK(HYPRE_ParVectorInitialize(one));
    CHECK(HYPRE_ParVectorSetConstantValues(one, 1.0));
  }
  CHECK(HYPRE_IJVectorCreate(HYPRE_COMM_SELF, 0, N - 1, &ib));
  CHECK(HYPRE_IJVectorSetObjectType(ib, HYPRE_PARCSR));
  CHECK(HYPRE_IJVectorInitialize(ib));
  CHECK(HYPRE_IJVectorAssemble(ib));
  CHECK(HYPRE_IJVectorGetObject(ib, (void **)&b));
  CHECK(HYPRE_ParCSRMatrixMatvec(1.0, A, one, 0.0, b)); /* b = A * 1 */
  CHECK(HYPRE_IJVectorCreate(HYPRE_COMM_SELF, 0, N - 1, &ix));
  CHECK(HYPRE_IJVectorSetObjectType(ix, HYPRE_PARCSR));
  CHECK(HYPRE_IJVectorInitialize(ix));
  CHECK(HYPRE_IJVectorAssemble(ix));
  CHECK(HYPRE_IJVectorGetObject(ix, (void **)&x));

  /* BoomerAMG as in ij -pmis -Pmx 0 -rlx 0 (ij.c:3365-3540 settings) */
  {
    HYPRE_Solver amg;
    CHECK(HYPRE_BoomerAMGCreate(&amg));
    CHECK(HYPRE_BoomerAMGSetMaxRowSum(amg, 1.0));
    CHECK(HYPRE_BoomerAMGSetStrongThreshold(amg, 0.25));
    CHECK(HYPRE_BoomerAMGSetTruncFactor(amg, 0.0));
    CHECK(HYPRE_BoomerAMGSetCoarsenType(amg, 8));
    CHECK(HYPRE_BoomerAMGSetInterpType(amg, 6));
    CHECK(HYPRE_BoomerAMGSetPMaxElmts(amg, 0));
    CHECK(HYPRE_BoomerAMGSetRelaxType(amg, 0));
    CHECK(HYPRE_BoomerAMGSetTol(amg, 1e-8));
    CHECK(HYPRE_BoomerAMGSetMaxIter(amg, 100));
    CHECK(HYPRE_BoomerAMGSetup(amg, A, b, x));
    CHECK(HYPRE_BoomerAMGSolve(amg, A, b, x));
    CHECK(HYPRE_BoomerAMGGetNumIterations(amg, &its));
    CHECK(HYPRE_BoomerAMGGetFinalRelativeResidualNorm(amg, &res));
    printf("amg %d %.6e\n", (int)its, res);
    CHECK(HYPRE_BoomerAMGDestroy(amg));
  }
  /* PCG preconditioned by one BoomerAMG V-cycle (ij -solver 1) */
  {
    HYPRE_Solver pcg, amg;
    CHECK(HYPRE_ParVectorSetConstantValues(x, 0.0));
    CHECK(HYPRE_ParCSRPCGCreate(HYPRE_COMM_SELF, &pcg));
    CHECK(HYPRE_ParCSRPCGSetTol(pcg, 1e-8));
    CHECK(HYPRE_ParCSRPCGSetMaxIter(pcg, 100));
    CHECK(HYPRE_ParCSRPCGSetTwoNorm(pcg, 1));
    CHECK(HYPRE_BoomerAMGCreate(&amg));
    CHECK(HYPRE_BoomerAMGSetMaxRowSum(amg, 1.0));
    CHECK(HYPRE_BoomerAMGSetPMaxElmts(amg, 4));
    CHECK(HYPRE_BoomerAMGSetTol(amg, 0.0));
    CHECK(HYPRE_BoomerAMGSetMaxIter(amg, 1));
    CHECK(HYPRE_ParCSRPCGSetPrecond(pcg, HYPRE_BoomerAMGSolve, HYPRE_BoomerAMGSetup, amg));
    CHECK(HYPRE_ParCSRPCGSetup(pcg, A, b, x));
    CHECK(HYPRE_ParCSRPCGSolve(pcg, A, b, x));
    CHECK(HYPRE_ParCSRPCGGetNumIterations(pcg, &its));
    CHECK(HYPRE_ParCSRPCGGetFinalRelativeResidualNorm(pcg, &res));
    printf("pcg %d %.6e\n", (int)its, res);
    CHECK(HYPRE_ParCSRPCGDestroy(pcg));
    CHECK(HYPRE_BoomerAMGDestroy(amg));
  }
  CHECK(HYPRE_IJVectorDestroy(ib));
  CHECK(HYPRE_IJVectorDestroy(ix));
  CHECK(HYPRE_ParVectorDestroy(one));
  CHECK(HYPRE_IJMatrixDestroy(ij));
  CHECK(HYPRE_Finalize());
  return 0;
}
