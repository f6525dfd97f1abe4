/*
 * hypre-ve_amd: MI355X-native BoomerAMG solve path behind hypre's C interface.
 *
 * Drop-in boundary: every entry point below has the name, argument meaning and
 * error behaviour of the reference's public function it replaces; the comment
 * on each cites the reference declaration (SX-Aurora/hypre-ve, src/...:line).
 * Plain C ABI: pointers and sizes only, no C++ or torch types.
 *
 * Memory model: HYPRE_ParVector / HYPRE_ParCSRMatrix data live in HBM
 * (HYPRE_MEMORY_DEVICE).  IJ set/get-values arrays are host arrays unless
 * HYPRE_SetMemoryLocation(HYPRE_MEMORY_DEVICE) was called, in which case they
 * are device pointers (reference: utilities/HYPRE_utilities.h, HYPRE_SetMemoryLocation).
 *
 * Communicator: the reference takes an MPI_Comm.  This build has no MPI; an
 * HYPRE_Comm is either HYPRE_COMM_SELF (one GPU) or a communicator created
 * by hypreve_CommCreate() over RCCL (one process per GPU).
 */
#ifndef HYPREVE_H
#define HYPREVE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* utilities/HYPRE_utilities.h: 32-bit ints, double reals (default build) */
typedef int HYPRE_Int;
typedef int HYPRE_BigInt;
typedef double HYPRE_Real;
typedef double HYPRE_Complex;

typedef struct hypreve_comm_struct *HYPRE_Comm;
#define HYPRE_COMM_SELF ((HYPRE_Comm)0)

typedef struct hypre_Solver_struct *HYPRE_Solver;
typedef struct hypre_ParCSRMatrix_struct *HYPRE_ParCSRMatrix;
typedef struct hypre_ParVector_struct *HYPRE_ParVector;
typedef struct hypre_IJMatrix_struct *HYPRE_IJMatrix;
typedef struct hypre_IJVector_struct *HYPRE_IJVector;

/* krylov/HYPRE_krylov.h:70 */
typedef HYPRE_Int (*HYPRE_PtrToParSolverFcn)(HYPRE_Solver, HYPRE_ParCSRMatrix, HYPRE_ParVector,
                                             HYPRE_ParVector);

#define HYPRE_PARCSR 5555          /* IJ_mv/HYPRE_IJ_mv.h object type */
#define HYPRE_MEMORY_HOST 0
#define HYPRE_MEMORY_DEVICE 1

/* error codes: utilities/HYPRE_utilities.h:80-86 */
#define HYPRE_ERROR_GENERIC 1
#define HYPRE_ERROR_MEMORY 2
#define HYPRE_ERROR_ARG 4
#define HYPRE_ERROR_CONV 256

/* ---------------- utilities (utilities/HYPRE_utilities.h) ---------------- */
HYPRE_Int HYPRE_Init(void);                                   /* HYPRE_utilities.h: HYPRE_Init */
HYPRE_Int HYPRE_Finalize(void);                               /* HYPRE_utilities.h: HYPRE_Finalize */
HYPRE_Int HYPRE_SetMemoryLocation(HYPRE_Int memory_location); /* HYPRE_utilities.h */
HYPRE_Int HYPRE_GetError(void);                               /* HYPRE_utilities.h: HYPRE_GetError */
HYPRE_Int HYPRE_ClearAllErrors(void);
HYPRE_Int HYPRE_CheckError(HYPRE_Int hypre_ierr, HYPRE_Int hypre_error_code);

/* ---------------- IJ interface (IJ_mv/HYPRE_IJ_mv.h) ---------------- */
HYPRE_Int HYPRE_IJMatrixCreate(HYPRE_Comm comm, HYPRE_BigInt ilower, HYPRE_BigInt iupper,
                               HYPRE_BigInt jlower, HYPRE_BigInt jupper,
                               HYPRE_IJMatrix *matrix);                       /* :68 */
HYPRE_Int HYPRE_IJMatrixDestroy(HYPRE_IJMatrix matrix);                       /* :80 */
HYPRE_Int HYPRE_IJMatrixInitialize(HYPRE_IJMatrix matrix);                    /* :90 */
HYPRE_Int HYPRE_IJMatrixSetObjectType(HYPRE_IJMatrix matrix, HYPRE_Int type); /* :235 */
HYPRE_Int HYPRE_IJMatrixSetValues(HYPRE_IJMatrix matrix, HYPRE_Int nrows, HYPRE_Int *ncols,
                                  const HYPRE_BigInt *rows, const HYPRE_BigInt *cols,
                                  const HYPRE_Complex *values);               /* :127 */
HYPRE_Int HYPRE_IJMatrixAddToValues(HYPRE_IJMatrix matrix, HYPRE_Int nrows, HYPRE_Int *ncols,
                                    const HYPRE_BigInt *rows, const HYPRE_BigInt *cols,
                                    const HYPRE_Complex *values);             /* :180 */
HYPRE_Int HYPRE_IJMatrixAssemble(HYPRE_IJMatrix matrix);                      /* :200 */
HYPRE_Int HYPRE_IJMatrixGetObject(HYPRE_IJMatrix matrix, void **object);      /* :259 */

HYPRE_Int HYPRE_IJVectorCreate(HYPRE_Comm comm, HYPRE_BigInt jlower, HYPRE_BigInt jupper,
                               HYPRE_IJVector *vector);                       /* :368 */
HYPRE_Int HYPRE_IJVectorDestroy(HYPRE_IJVector vector);                       /* :378 */
HYPRE_Int HYPRE_IJVectorInitialize(HYPRE_IJVector vector);                    /* :386 */
HYPRE_Int HYPRE_IJVectorSetObjectType(HYPRE_IJVector vector, HYPRE_Int type);
HYPRE_Int HYPRE_IJVectorSetValues(HYPRE_IJVector vector, HYPRE_Int nvalues,
                                  const HYPRE_BigInt *indices,
                                  const HYPRE_Complex *values);               /* :423 */
HYPRE_Int HYPRE_IJVectorGetValues(HYPRE_IJVector vector, HYPRE_Int nvalues,
                                  const HYPRE_BigInt *indices, HYPRE_Complex *values); /* :453 */
HYPRE_Int HYPRE_IJVectorAssemble(HYPRE_IJVector vector);
HYPRE_Int HYPRE_IJVectorGetObject(HYPRE_IJVector vector, void **object);

/* ---------------- ParCSR (parcsr_mv/HYPRE_parcsr_mv.h) ---------------- */
HYPRE_Int HYPRE_ParCSRMatrixDestroy(HYPRE_ParCSRMatrix matrix);
HYPRE_Int HYPRE_ParCSRMatrixGetLocalRange(HYPRE_ParCSRMatrix matrix, HYPRE_BigInt *row_start,
                                          HYPRE_BigInt *row_end, HYPRE_BigInt *col_start,
                                          HYPRE_BigInt *col_end);
/* :51  y = alpha*A*x + beta*y, on the GPU */
HYPRE_Int HYPRE_ParCSRMatrixMatvec(HYPRE_Complex alpha, HYPRE_ParCSRMatrix A, HYPRE_ParVector x,
                                   HYPRE_Complex beta, HYPRE_ParVector y);
/* parcsr_mv/protos: hypre_ParCSRMatrixMatvecOutOfPlace  y = alpha*A*x + beta*b */
HYPRE_Int HYPRE_ParCSRMatrixMatvecOutOfPlace(HYPRE_Complex alpha, HYPRE_ParCSRMatrix A,
                                             HYPRE_ParVector x, HYPRE_Complex beta,
                                             HYPRE_ParVector b, HYPRE_ParVector y);
HYPRE_Int HYPRE_ParCSRMatrixMatvecT(HYPRE_Complex alpha, HYPRE_ParCSRMatrix A, HYPRE_ParVector x,
                                    HYPRE_Complex beta, HYPRE_ParVector y);
HYPRE_Int HYPRE_ParVectorCreate(HYPRE_Comm comm, HYPRE_BigInt global_size,
                                HYPRE_BigInt *partitioning, HYPRE_ParVector *vector);
HYPRE_Int HYPRE_ParVectorInitialize(HYPRE_ParVector vector);
HYPRE_Int HYPRE_ParVectorDestroy(HYPRE_ParVector vector);
HYPRE_Int HYPRE_ParVectorSetConstantValues(HYPRE_ParVector vector, HYPRE_Complex value);
HYPRE_Int HYPRE_ParVectorCopy(HYPRE_ParVector x, HYPRE_ParVector y);
HYPRE_Int HYPRE_ParVectorScale(HYPRE_Complex value, HYPRE_ParVector x);
HYPRE_Int HYPRE_ParVectorAxpy(HYPRE_Complex alpha, HYPRE_ParVector x, HYPRE_ParVector y);
HYPRE_Int HYPRE_ParVectorInnerProd(HYPRE_ParVector x, HYPRE_ParVector y, HYPRE_Real *prod); /* :64 */

/* ---------------- generators (parcsr_ls/HYPRE_parcsr_ls.h) ---------------- */
/* :4168 GenerateLaplacian (value[0..3] = diag, -cx, -cy, -cz); this rank owns
 * grid block (p,q,r) of a P x Q x R process grid. */
HYPRE_ParCSRMatrix GenerateLaplacian(HYPRE_Comm comm, HYPRE_BigInt nx, HYPRE_BigInt ny,
                                     HYPRE_BigInt nz, HYPRE_Int P, HYPRE_Int Q, HYPRE_Int R,
                                     HYPRE_Int p, HYPRE_Int q, HYPRE_Int r, HYPRE_Real *value);
/* :4180 GenerateLaplacian27pt */
HYPRE_ParCSRMatrix GenerateLaplacian27pt(HYPRE_Comm comm, HYPRE_BigInt nx, HYPRE_BigInt ny,
                                         HYPRE_BigInt nz, HYPRE_Int P, HYPRE_Int Q, HYPRE_Int R,
                                         HYPRE_Int p, HYPRE_Int q, HYPRE_Int r, HYPRE_Real *value);

/* ---------------- BoomerAMG (parcsr_ls/HYPRE_parcsr_ls.h) ---------------- */
HYPRE_Int HYPRE_BoomerAMGCreate(HYPRE_Solver *solver);                          /* :83 */
HYPRE_Int HYPRE_BoomerAMGDestroy(HYPRE_Solver solver);                          /* :89 */
HYPRE_Int HYPRE_BoomerAMGSetup(HYPRE_Solver solver, HYPRE_ParCSRMatrix A, HYPRE_ParVector b,
                               HYPRE_ParVector x);                              /* :100 */
HYPRE_Int HYPRE_BoomerAMGSolve(HYPRE_Solver solver, HYPRE_ParCSRMatrix A, HYPRE_ParVector b,
                               HYPRE_ParVector x);                              /* :115 */
HYPRE_Int HYPRE_BoomerAMGGetNumIterations(HYPRE_Solver solver, HYPRE_Int *num_iterations); /* :155 */
HYPRE_Int HYPRE_BoomerAMGGetFinalRelativeResidualNorm(HYPRE_Solver solver, HYPRE_Real *rel_resid_norm); /* :161 */
HYPRE_Int HYPRE_BoomerAMGSetConvergeType(HYPRE_Solver solver, HYPRE_Int type);  /* :184 */
HYPRE_Int HYPRE_BoomerAMGSetTol(HYPRE_Solver solver, HYPRE_Real tol);           /* :192 */
HYPRE_Int HYPRE_BoomerAMGSetMaxIter(HYPRE_Solver solver, HYPRE_Int max_iter);   /* :200 */
HYPRE_Int HYPRE_BoomerAMGSetMinIter(HYPRE_Solver solver, HYPRE_Int min_iter);   /* :206 */
HYPRE_Int HYPRE_BoomerAMGSetMaxCoarseSize(HYPRE_Solver solver, HYPRE_Int max_coarse_size); /* :213 */
HYPRE_Int HYPRE_BoomerAMGSetMinCoarseSize(HYPRE_Solver solver, HYPRE_Int min_coarse_size); /* :220 */
HYPRE_Int HYPRE_BoomerAMGSetMaxLevels(HYPRE_Solver solver, HYPRE_Int max_levels);  /* :227 */
HYPRE_Int HYPRE_BoomerAMGSetStrongThreshold(HYPRE_Solver solver, HYPRE_Real strong_threshold); /* :246 */
HYPRE_Int HYPRE_BoomerAMGSetMaxRowSum(HYPRE_Solver solver, HYPRE_Real max_row_sum); /* :283 */
HYPRE_Int HYPRE_BoomerAMGSetCoarsenType(HYPRE_Solver solver, HYPRE_Int coarsen_type); /* :310; 8 PMIS, 9 PMIS (no random), 10 HMIS, 11 Ruge first pass */
HYPRE_Int HYPRE_BoomerAMGSetMeasureType(HYPRE_Solver solver, HYPRE_Int measure_type); /* :362 */
HYPRE_Int HYPRE_BoomerAMGSetAggNumLevels(HYPRE_Solver solver, HYPRE_Int agg_num_levels); /* :369 */
HYPRE_Int HYPRE_BoomerAMGSetNumPaths(HYPRE_Solver solver, HYPRE_Int num_paths); /* :377 */
/* Aggressive-level interpolation: 4 (multipass, the default), 5 (2-stage
 * extended, matrix-matrix form: par_mod_lr_interp.c:16 then par_2s_interp.c:15),
 * 7 (2-stage extended+e: par_mod_lr_interp.c:1040 then par_2s_interp.c:564),
 * 1 / 3 (2-stage extended+i / extended, then partial.c:16 / :1855), 2 (standard,
 * then partial standard, partial.c:859) and 6 (MM extended+i, then partial
 * extended+i); Setup fails with HYPRE_ERROR_ARG for 8. */
HYPRE_Int HYPRE_BoomerAMGSetAggInterpType(HYPRE_Solver solver, HYPRE_Int agg_interp_type); /* :480 */
HYPRE_Int HYPRE_BoomerAMGSetAggTruncFactor(HYPRE_Solver solver, HYPRE_Real agg_trunc_factor); /* :488 */
HYPRE_Int HYPRE_BoomerAMGSetAggP12TruncFactor(HYPRE_Solver solver, HYPRE_Real agg_P12_trunc_factor); /* :496 */
HYPRE_Int HYPRE_BoomerAMGSetAggPMaxElmts(HYPRE_Solver solver, HYPRE_Int agg_P_max_elmts); /* :504 */
HYPRE_Int HYPRE_BoomerAMGSetAggP12MaxElmts(HYPRE_Solver solver, HYPRE_Int agg_P12_max_elmts); /* :512 */
/* interp_type 6 ext+i, 14 ext, 16 / 17 / 18 ext / ext+i / ext+e (matrix-matrix form), 3 direct,
 * 7 ext+i where no common C point, 8 / 9 standard (9: separated weights) */
HYPRE_Int HYPRE_BoomerAMGSetInterpType(HYPRE_Solver solver, HYPRE_Int interp_type); /* :442 */
HYPRE_Int HYPRE_BoomerAMGSetSepWeight(HYPRE_Solver solver, HYPRE_Int sep_weight); /* :464 (standard interpolation) */
/* :667 / :673: redundant coarse-grid AMG below seq_threshold global rows; it
 * acts only with more than one rank, as in the reference (par_amg_setup.c:294):
 * under hypreve_BoomerAMGSetRankEmulation, and on N ranks (the rank-0
 * gathered setup runs that emulation) */
HYPRE_Int HYPRE_BoomerAMGSetSeqThreshold(HYPRE_Solver solver, HYPRE_Int seq_threshold);
/* :168: systems AMG, unknown approach (interleaved functions, dof = row %
 * num_functions; strength and weak lumping within a function); with
 * interp_type 6 / 14 and agg_interp_type 1 / 3 / 4, one-process setup */
HYPRE_Int HYPRE_BoomerAMGSetNumFunctions(HYPRE_Solver solver, HYPRE_Int num_functions);
HYPRE_Int HYPRE_BoomerAMGSetDofFunc(HYPRE_Solver solver, HYPRE_Int *dof_func); /* :176 (read at Setup; one process) */
HYPRE_Int HYPRE_BoomerAMGSetRedundant(HYPRE_Solver solver, HYPRE_Int redundant);
HYPRE_Int HYPRE_BoomerAMGSetTruncFactor(HYPRE_Solver solver, HYPRE_Real trunc_factor); /* :448 */
HYPRE_Int HYPRE_BoomerAMGSetPMaxElmts(HYPRE_Solver solver, HYPRE_Int P_max_elmts); /* :455 */
HYPRE_Int HYPRE_BoomerAMGSetCycleType(HYPRE_Solver solver, HYPRE_Int cycle_type); /* :572 */
HYPRE_Int HYPRE_BoomerAMGSetNumSweeps(HYPRE_Solver solver, HYPRE_Int num_sweeps); /* :691 */
HYPRE_Int HYPRE_BoomerAMGSetCycleNumSweeps(HYPRE_Solver solver, HYPRE_Int num_sweeps, HYPRE_Int k); /* :702 */
HYPRE_Int HYPRE_BoomerAMGSetRelaxType(HYPRE_Solver solver, HYPRE_Int relax_type); /* :741; 0, 3/4/6/8/13/14, 7, 16, 17 (FCF-Jacobi), 18; coarsest 9 */
HYPRE_Int HYPRE_BoomerAMGSetCycleRelaxType(HYPRE_Solver solver, HYPRE_Int relax_type, HYPRE_Int k); /* :753 */
HYPRE_Int HYPRE_BoomerAMGSetRelaxOrder(HYPRE_Solver solver, HYPRE_Int relax_order); /* :770 */
HYPRE_Int HYPRE_BoomerAMGSetRelaxWt(HYPRE_Solver solver, HYPRE_Real relax_weight); /* :805 */
HYPRE_Int HYPRE_BoomerAMGSetOuterWt(HYPRE_Solver solver, HYPRE_Real omega);       /* :839 */
HYPRE_Int HYPRE_BoomerAMGSetLevelRelaxWt(HYPRE_Solver solver, HYPRE_Real relax_weight,
                                         HYPRE_Int level);                          /* :815 */
HYPRE_Int HYPRE_BoomerAMGSetLevelOuterWt(HYPRE_Solver solver, HYPRE_Real omega,
                                         HYPRE_Int level);                          /* :849 */
HYPRE_Int HYPRE_BoomerAMGSetPrintLevel(HYPRE_Solver solver, HYPRE_Int print_level); /* :1103 */
/* Chebyshev smoother (relax type 16), HYPRE_parcsr_ls.h:857-889 */
HYPRE_Int HYPRE_BoomerAMGSetChebyOrder(HYPRE_Solver solver, HYPRE_Int order);          /* :857 */
HYPRE_Int HYPRE_BoomerAMGSetChebyFraction(HYPRE_Solver solver, HYPRE_Real ratio);      /* :864 */
HYPRE_Int HYPRE_BoomerAMGSetChebyScale(HYPRE_Solver solver, HYPRE_Int scale);          /* :871 */
HYPRE_Int HYPRE_BoomerAMGSetChebyVariant(HYPRE_Solver solver, HYPRE_Int variant);      /* :878 */
HYPRE_Int HYPRE_BoomerAMGSetChebyEigEst(HYPRE_Solver solver, HYPRE_Int eig_est);       /* :889 */
HYPRE_Int HYPRE_BoomerAMGSetLogging(HYPRE_Solver solver, HYPRE_Int logging);
HYPRE_Int HYPRE_BoomerAMGGetNumLevels(HYPRE_Solver solver, HYPRE_Int *num_levels);

/* ---------------- PCG (parcsr_ls/HYPRE_parcsr_ls.h, krylov/HYPRE_krylov.h) ------- */
HYPRE_Int HYPRE_ParCSRPCGCreate(HYPRE_Comm comm, HYPRE_Solver *solver);        /* :2403 */
HYPRE_Int HYPRE_ParCSRPCGDestroy(HYPRE_Solver solver);                          /* :2409 */
HYPRE_Int HYPRE_ParCSRPCGSetup(HYPRE_Solver solver, HYPRE_ParCSRMatrix A, HYPRE_ParVector b,
                               HYPRE_ParVector x);                              /* :2411 */
HYPRE_Int HYPRE_ParCSRPCGSolve(HYPRE_Solver solver, HYPRE_ParCSRMatrix A, HYPRE_ParVector b,
                               HYPRE_ParVector x);                              /* :2416 */
HYPRE_Int HYPRE_ParCSRPCGSetTol(HYPRE_Solver solver, HYPRE_Real tol);           /* :2421 */
HYPRE_Int HYPRE_ParCSRPCGSetMaxIter(HYPRE_Solver solver, HYPRE_Int max_iter);   /* :2427 */
HYPRE_Int HYPRE_ParCSRPCGSetTwoNorm(HYPRE_Solver solver, HYPRE_Int two_norm);   /* :2436 */
HYPRE_Int HYPRE_ParCSRPCGSetPrecond(HYPRE_Solver solver, HYPRE_PtrToParSolverFcn precond,
                                    HYPRE_PtrToParSolverFcn precond_setup,
                                    HYPRE_Solver precond_solver);               /* :2442 */
HYPRE_Int HYPRE_ParCSRPCGSetPrintLevel(HYPRE_Solver solver, HYPRE_Int level);  /* :2453 */
HYPRE_Int HYPRE_ParCSRPCGGetNumIterations(HYPRE_Solver solver, HYPRE_Int *num_iterations); /* :2456 */
HYPRE_Int HYPRE_ParCSRPCGGetFinalRelativeResidualNorm(HYPRE_Solver solver, HYPRE_Real *norm); /* :2459 */

/* ---------------- hypre-ve_amd extensions (no reference counterpart) ------------ */
/* Communicator over RCCL: rank/size of this process, nccl_id = 128-byte
 * ncclUniqueId produced on rank 0 by hypreve_CommGetUniqueId and broadcast by
 * the caller (torch.distributed, MPI, a file...). */
HYPRE_Int hypreve_CommGetUniqueId(void *nccl_id_128);
HYPRE_Int hypreve_CommCreate(HYPRE_Int rank, HYPRE_Int size, const void *nccl_id_128,
                             HYPRE_Comm *comm);
HYPRE_Int hypreve_CommDestroy(HYPRE_Comm comm);
/* Transport self-test (collective): grouped exchange with every rank, self
 * included, all-reduce, all-gather and broadcast, each checked.  0 = pass.
 * hypreve_CommCreate with size 1 and an id makes a 1-rank RCCL communicator,
 * which runs the partitioned solve path with one rank. */
HYPRE_Int hypreve_CommSelfTest(HYPRE_Comm comm);
/* `size` communicators of virtual ranks sharing one GPU inside this process
 * (comms[0..size-1]); each rank must be driven from its own host thread.  Used
 * to check the partitioned solve on a single GPU (RCCL refuses two ranks on
 * one device); not a production transport. */
HYPRE_Int hypreve_CommCreateLoopback(HYPRE_Int size, HYPRE_Comm *comms);
/* Communicator of `size` processes on one host over the POSIX shared-memory
 * segment `shm_name` (rank 0 creates and finally unlinks it; every rank passes
 * the same name).  Host-staged: each exchange drains the stream and copies
 * through host memory.  It lets several processes share one GPU, which RCCL
 * refuses, so the process-per-rank path can be tested on a one-GPU box; not a
 * production transport. */
HYPRE_Int hypreve_CommCreateShm(HYPRE_Int rank, HYPRE_Int size, const char *shm_name, HYPRE_Comm *comm);

/* Direct construction of a local ParCSR block from host CSR arrays (global
 * column indices), equivalent to IJ create/set/assemble in one call. */
HYPRE_Int hypreve_ParCSRMatrixCreateFromCSR(HYPRE_Comm comm, HYPRE_BigInt first_row,
                                            HYPRE_Int local_rows, HYPRE_BigInt global_rows,
                                            const HYPRE_Int *row_ptr, const HYPRE_BigInt *cols,
                                            const HYPRE_Real *vals, HYPRE_ParCSRMatrix *A);
/* Device pointer / length of a vector's local part (for zero-copy use). */
HYPRE_Real *hypreve_ParVectorDeviceData(HYPRE_ParVector v);
HYPRE_Int hypreve_ParVectorLocalSize(HYPRE_ParVector v);
HYPRE_Int hypreve_ParVectorCopyToHost(HYPRE_ParVector v, HYPRE_Real *host);
HYPRE_Int hypreve_ParVectorCopyFromHost(HYPRE_ParVector v, const HYPRE_Real *host);
HYPRE_Int hypreve_ParVectorSetRandomValues(HYPRE_ParVector v, HYPRE_Int seed); /* HYPRE_ParVectorSetRandomValues */

/* Number of contiguous row blocks used by the hybrid Gauss-Seidel smoothers
 * (reference: OMP_NUM_THREADS on the CPU path). 0 = automatic (the default):
 * one block per 4096 local level-0 rows, resolved at Setup; 1 reproduces the
 * reference's single-thread sweep. */
HYPRE_Int hypreve_BoomerAMGSetNumBlocks(HYPRE_Solver solver, HYPRE_Int num_blocks);
/* Tuning: visit the row blocks of every operator in nbands bands of the grid
 * (0 = natural order) on the built hierarchy; results are unchanged. */
HYPRE_Int hypreve_BoomerAMGSetBlockBands(HYPRE_Solver solver, HYPRE_Int nbands,
                                         HYPRE_Int which_mask); /* bit 0 A, 1 P, 2 R (0 = all) */
/* Device layout / row loop of the hierarchy's SELL operators (takes effect at
 * Setup): 0 automatic, 1 padded lane-per-row, 2 jagged lane-per-row, 3 padded
 * workgroup-per-slice, 4 jagged wave-product-parallel, 5 jagged with an LDS
 * x-tile (per-slice column dictionary), 6 padded with 16-bit column deltas
 * against per-slot bases (where a slice's rows fit), 7 as 6 plus 8-bit value
 * indices into a table of the operator's distinct values (where at most 256
 * occur), 8 padded and 9 jagged, each with 16-bit value indices (where at
 * most 4096 distinct values occur), 10 jagged with an LDS x-tile made of at
 * most 63 contiguous column ranges (range dictionary), 11 slot-uniform
 * stencil layout (per slice and slot one column offset, one value and a lane
 * mask; nothing stored per entry) where an operator is a constant-coefficient
 * stencil, else as 7, 12 offset-coded P and R (one 16-bit code per entry:
 * offset from the row's grid point and value index) where they build, else
 * padded, 13 packed P and R (one 32-bit code per entry: column less the
 * slice's smallest column, and value index) where they fit, else as 8,
 * 14 as 5 with the per-entry streams (5 and the automatic choice store the
 * dictionary layout's values and columns lane-packed, 16 B a lane load),
 * 15 as 12 with R in the jagged, product-parallel coded form (the automatic
 * choice for restrictions; 12 keeps them padded).
 * All give identical bits; the forced settings exist for parity tests
 * and experiments. */
HYPRE_Int hypreve_BoomerAMGSetSellPolicy(HYPRE_Solver solver, HYPRE_Int policy);
/* One GPU runs the hybrid Gauss-Seidel smoothers with the row blocks of an
 * N-rank run whose level-0 rows start at starts[0..nranks] (num_blocks blocks
 * of each rank's rows on every level, par_relax.c's per-process thread blocks;
 * l1 norms to match), so its iterates equal the N-rank iterates. nranks <= 1
 * clears it. Takes effect at Setup. */
HYPRE_Int hypreve_BoomerAMGSetGsRankStarts(HYPRE_Solver solver, HYPRE_Int nranks, const HYPRE_Int *starts);
/* The relaxation weight and outer weight (omega) the cycle uses on `level`. */
HYPRE_Int hypreve_BoomerAMGGetLevelWeights(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Real *relax_weight,
                                           HYPRE_Real *omega);
/* HMIS (coarsen_type 10) on one process as an N-rank run's setup coarsens
 * it: each rank's Ruge first pass over the strong connections it owns and a
 * random stream per rank in the PMIS stage (par_coarsen.c:2774 on N
 * processes), rank r owning level-0 rows starts[r] .. starts[r+1]-1 and the
 * C points of its rows below.  The rest of the setup stays the one-process
 * one (a partial emulation, for experiments; an N-rank setup follows the
 * whole of hypreve_BoomerAMGSetRankEmulation).  nranks <= 1 clears it; other
 * coarsenings ignore it.  Takes effect at Setup. */
HYPRE_Int hypreve_BoomerAMGSetCoarsenRankStarts(HYPRE_Solver solver, HYPRE_Int nranks, const HYPRE_Int *starts);
/* One process reproduces the setup and smoothing of a reference N-rank run
 * (mpirun -np N) whose level-0 rows start at starts[0..nranks]: every row in
 * ParCSR order (the rank's own columns, then the others; par_csr_matrix.c),
 * per-rank PMIS random streams (par_indepset.c:25, seed 2747 + rank), per-rank
 * HMIS first passes (par_coarsen.c:874 on S_diag), the CF_marker_offd
 * semantics of par_coarsen.c:2296/2348, truncation over [P_diag | P_offd]
 * (par_csr_matrix.c:2671), and the hybrid GS blocks of SetGsRankStarts.
 * Coarse-level agglomeration is off (the reference has none).  This pins the
 * product to the reference's own np > 1 saved outputs.  nranks <= 1 clears it.
 * Interpolation: ext+i (6) and ext (14) per rank, the matrix-matrix forms
 * (16 / 17 / 18) with hypre_ParMatmul's np > 1 entry order; aggressive levels:
 * the second pass per rank as well, multipass rows in P_diag | P_offd order,
 * and the 2-stage types.  These are the rules of every N-rank setup of this
 * library too (the distributed one, dsetup.cpp, and the rank-0 gathered one),
 * so an N-GPU run equals a one-GPU run given the same starts here bit for
 * bit, and both reproduce the reference's N-process run.  Takes effect at
 * Setup. */
HYPRE_Int hypreve_BoomerAMGSetRankEmulation(HYPRE_Solver solver, HYPRE_Int nranks, const HYPRE_Int *starts);
/* Multi-rank: coarse levels with at most `rows` global rows (from the first
 * such level down) are held whole by every rank and cycled redundantly, with
 * one all-gather on the way down instead of halo exchanges on every coarse
 * level (same bits).  0 = never; < 0 (the default): automatic, from the first
 * level with at most 12288 rows per rank. */
HYPRE_Int hypreve_BoomerAMGSetAggloRows(HYPRE_Solver solver, HYPRE_Int rows);
/* Whole-cycle hipGraph capture on/off (default on). */
HYPRE_Int hypreve_BoomerAMGSetUseGraph(HYPRE_Solver solver, HYPRE_Int use_graph);
/* Statistics after Setup: levels, complexities, per-level rows/nnz. */
HYPRE_Int hypreve_BoomerAMGGetComplexities(HYPRE_Solver solver, HYPRE_Real *grid,
                                           HYPRE_Real *oper, HYPRE_Real *cycle);
HYPRE_Int hypreve_BoomerAMGGetLevelInfo(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int *rows,
                                        int64_t *nnz_A, int64_t *nnz_P);
/* Export one level of the (host-side) hierarchy for inspection/testing.
 * which: 0 = A, 1 = P, 2 = R = P^T.  Pass NULL arrays to query sizes. */
HYPRE_Int hypreve_BoomerAMGGetLevelMatrix(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int which,
                                          HYPRE_Int *nrows, HYPRE_Int *ncols, int64_t *nnz,
                                          HYPRE_Int *row_ptr, HYPRE_Int *cols, HYPRE_Real *vals);
HYPRE_Int hypreve_BoomerAMGGetLevelVector(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int which,
                                          HYPRE_Int *n, void *data); /* 0 cf (int), 1 l1, 2 Chebyshev ds (double),
                                                                        3 hybrid-GS block starts of the N-rank emulation (int) */
/* Chebyshev data of one level: coefficient count / values (up to 5), the
 * eigenvalue estimates eig[0] = max, eig[1] = min, and params[0..2] = order,
 * scale, variant. */
HYPRE_Int hypreve_BoomerAMGGetChebyInfo(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int *ncoefs,
                                        HYPRE_Real *coefs, HYPRE_Real *eig, HYPRE_Int *params);
HYPRE_Int hypreve_BoomerAMGGetCoarseMatrix(HYPRE_Solver solver, HYPRE_Int *n, HYPRE_Real *dense);
HYPRE_Int hypreve_BoomerAMGGetRelaxInfo(HYPRE_Solver solver, HYPRE_Int *relax_type4,
                                        HYPRE_Int *num_sweeps4, HYPRE_Real *weights2,
                                        HYPRE_Int *misc4); /* misc: relax_order, cycle_type, num_blocks,
                                                               user relax type (-1: unset) */
/* Host-only setup (no device upload): lets the CPU test suite check the
 * hierarchy against the reference fixtures on a machine without a GPU. */
HYPRE_Int hypreve_BoomerAMGSetupHost(HYPRE_Solver solver, HYPRE_ParCSRMatrix A);
/* CPU self-check of the row partition of the host hierarchy over `size`
 * ranks: reassembly, pairwise halo plans, emulated distributed apply. */
HYPRE_Int hypreve_BoomerAMGPartitionCheck(HYPRE_Solver solver, HYPRE_Int size);
/* CPU self-check of the distributed setup: the one-process matrix A split in
 * `size` row blocks, set up by `size` host threads exchanging ghost rows,
 * against the one-process setup partitioned the same way (bytewise). */
HYPRE_Int hypreve_BoomerAMGDistSetupCheck(HYPRE_Solver solver, HYPRE_ParCSRMatrix A, HYPRE_Int size);
/* Run exactly one cycle (hypre_BoomerAMGCycle) on device vectors f, u. */
HYPRE_Int hypreve_BoomerAMGCycle(HYPRE_Solver solver, HYPRE_ParVector f, HYPRE_ParVector u);
/* Device timing of the last Solve, per kernel class (ms), for bench/profiling. */
HYPRE_Int hypreve_BoomerAMGGetKernelStats(HYPRE_Solver solver, HYPRE_Real *stats, HYPRE_Int n);
/* Time `reps` launches of the finest-level residual SpMV r = b - A x with HIP
 * events on the solver's stream; returns avg ms and the algorithmic bytes. */
HYPRE_Int hypreve_BenchFineSpMV(HYPRE_Solver solver, HYPRE_Int reps, HYPRE_Real *avg_ms,
                                HYPRE_Real *bytes);
/* Bytes the same launch streams in the stored layout (padding, 16-bit column
 * deltas and slot bases included) plus its three vectors. */
HYPRE_Int hypreve_BenchFineSpMVStoredBytes(HYPRE_Solver solver, HYPRE_Real *bytes);
/* Device layout of a level operator's interior rows (which: 0 A, 1 P, 2 R):
 * 0 padded SELL-64, 1 jagged, 2 workgroup-per-slice, 3 jagged wave-product,
 * 4 dictionary, 5 16-bit column deltas, 6 deltas + 8-bit value table,
 * 7 deltas + 16-bit value table, 8 padded + 16-bit value table, 9 jagged +
 * 16-bit value table, 10 range dictionary, 11 slot-uniform stencil,
 * 12 offset-coded (P, R), 13 packed 32-bit codes (P, R), 14 slot-uniform
 * stencil over a grid in natural order (k_grid_stencil: LDS x-tile),
 * 15 dictionary with lane-packed value / column streams (k_sell_dictw),
 * 16 offset-coded, jagged and product-parallel (k_code_pw: R). */
HYPRE_Int hypreve_BoomerAMGGetLevelLayout(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int which, HYPRE_Int *kind);
/* Host check: each hybrid Gauss-Seidel level schedule (num_blocks row blocks)
 * reproduces the sequential per-block sweep bit for bit on random data. */
HYPRE_Int hypreve_BoomerAMGGsScheduleCheck(HYPRE_Solver solver, HYPRE_Int num_blocks);
/* This rank's communication in one V-cycle (the last one run), level `level`:
 * out[5] = {halo exchanges, bytes they send, all-gathers into the replicated
 * levels, their bytes sent, all-reduces}; zeros on one rank. */
HYPRE_Int hypreve_BoomerAMGGetCycleCommStats(HYPRE_Solver solver, HYPRE_Int level, int64_t *out);
/* Size of the packed hybrid Gauss-Seidel schedule of level `level`'s A with
 * num_blocks blocks (host only, after Setup / SetupHost): out[6] = {nnz, stored
 * entries, steps, teams, longest team in steps, blocks}. */
HYPRE_Int hypreve_BoomerAMGGsScheduleStats(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int forward,
                                           HYPRE_Int num_blocks, int64_t *out);
/* Host check of the slot-uniform stencil layout of level's A (after
 * hypreve_BoomerAMGSetupHost or Setup): every row rebuilt from its slice's
 * slot pattern equals the CSR row entry for entry.  *width = 0 (and
 * *npatterns = 0) when the operator is not a constant-coefficient stencil. */
HYPRE_Int hypreve_BoomerAMGStencilLayoutCheck(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int *width,
                                              HYPRE_Int *npatterns);
/* 1 when the grid-stencil loop (k_grid_stencil: 32-bit buffer byte offsets)
 * can address an nx x ny x nz grid on one rank, else 0: a larger rank share
 * keeps the per-slice stencil loop (no GPU needed). */
HYPRE_Int hypreve_GridStencilAddressable(HYPRE_BigInt nx, HYPRE_BigInt ny, HYPRE_BigInt nz);
/* Setup's heavy row loops on the GPU (default 1): strength and PMIS
 * coarsening (one process, coarsen_type 8 / 9, levels of 2^16 rows and more),
 * ext+i interpolation and its truncation, R = P^T and the Galerkin product
 * RAP, byte for byte the host functions' result (device/setup_dev.hip); 0 runs
 * them on the host.  The distributed setup keeps the host. */
HYPRE_Int hypreve_BoomerAMGSetDeviceSetup(HYPRE_Solver solver, HYPRE_Int on);
/* The setup's log (levels, phase times, rows the device setup left to the
 * host) into buf[0..len). */
HYPRE_Int hypreve_BoomerAMGGetSetupLog(HYPRE_Solver solver, char *buf, HYPRE_Int len);
/* The path the last Setup took: 0 one process, 1 one process under
 * hypreve_BoomerAMGSetRankEmulation, 2 distributed (every rank its own rows,
 * hypre's N-process rules), 3 gathered on rank 0 under the rank emulation of
 * the same N-process rules (the options the distributed setup does not take),
 * 4 gathered one-process (direct interpolation, which the emulation does not
 * restate); -1 before the first Setup. */
HYPRE_Int hypreve_BoomerAMGGetSetupPath(HYPRE_Solver solver, HYPRE_Int *path);
/* Host check of the offset-coded layout of level's P (which 1) or R (which 2)
 * (after hypreve_BoomerAMGSetupHost or Setup): every row decoded from its
 * 16-bit codes equals the CSR row entry for entry, values bitwise.
 * *noffsets = *nvalues = 0 when the operator does not code in 16 bits. */
HYPRE_Int hypreve_BoomerAMGCodedLayoutCheck(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int which,
                                            HYPRE_Int *noffsets, HYPRE_Int *nvalues);
/* One level operator (which 0 = A as residual, 1 = P as prolongation, 2 = R
 * as restriction): average ms over reps, algorithmic bytes, padded entries. */
HYPRE_Int hypreve_BenchLevelOp(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int which, HYPRE_Int reps,
                               HYPRE_Real *avg_ms, HYPRE_Real *bytes, HYPRE_Real *padded_nnz);
/* Tuning harness: the matrix's rows uploaded alone in layout `policy` (0 =
 * automatic, as hypreve_BoomerAMGSetSellPolicy) with an nbands traversal, op
 * (0 residual, 1 matvec, 2 l1-Jacobi, 8 residual + l1-Jacobi with the norm
 * partials; the l1 forms take their norms on the fly, stencil / delta layouts)
 * applied reps times: average ms, bytes of the stored layout + 24 B a row,
 * and a layout description in layout[0..len). */
HYPRE_Int hypreve_BenchOperator(HYPRE_ParCSRMatrix A, HYPRE_Int op, HYPRE_Int policy, HYPRE_Int nbands,
                                HYPRE_Int reps, HYPRE_Real *avg_ms, HYPRE_Real *stored_bytes, char *layout,
                                HYPRE_Int len);
/* Tuning knobs read at kernel launch or setup (0 = built-in default): 0 row
 * blocks per step of the offset-coded loop (1, 2, 4), 1 its codes per batch
 * (4, 8, 16), 2 its persistent workgroups per CU (also the jagged coded
 * loop's), 3 the stream-mix access width (2: 16 B), 4 the jagged coded loop's
 * entries per row and chunk (4, 8, 16), 5 = 1 its code prefetch off, 6 = 1
 * the hybrid-GS sweep's unpaired entry loads, 7 the device setup's LDS table
 * cap (2^v slots; rows beyond it are finished on the host), 8 the pipelined
 * GS sweep on every schedule (1) or none (2), 9 the grid-stencil z-chunk,
 * 10 the pipelined GS sweep's unit capacity (128, 256, 512), 11 (tests) the
 * GS ring reach shortened, 12 = 256 the unpipelined GS sweep's chunk, 13 = 1
 * the GS scatter pass after the sweep, 14 = 16 (setup) 16-lane GS ring slots
 * for the wide operators, 15 (setup) the smallest level the device strength
 * and PMIS take, 16 the GS sweeps' LDS pad a workgroup in KiB (-1: none), 17
 * extra LDS a workgroup of the dictionary loops in KiB, 19 (setup) the log2
 * size of the small tables of the ext+i and RAP fills.  Ids 0-31.  Results
 * are unchanged, except knob 11's, which gs_schedule_self_check must
 * refuse. */
HYPRE_Int hypreve_SetKnob(HYPRE_Int id, HYPRE_Int value);
/* Bytes the same launch streams in the operator's stored (compressed) layout,
 * vectors included. */
HYPRE_Int hypreve_BenchLevelOpStoredBytes(HYPRE_Solver solver, HYPRE_Int level, HYPRE_Int which,
                                          HYPRE_Real *bytes);
/* Read-only streaming kernel (elem_bytes 2, 4, 8 or 16): FETCH_SIZE calibration.
 * elem_bytes -1 / -2 / -5: a read/write mix, R = 1, 2 or 5 streams of n doubles
 * read and one written per element (the achievable bandwidth of a kernel that
 * reads R bytes for each byte it writes).  elem_bytes -8: n doubles read as
 * per-wave contiguous 16 KiB segments (the row loops' access shape); -9: the
 * same with the 4 waves of a workgroup interleaved over 512-B chunks. */
HYPRE_Int hypreve_BenchStream(HYPRE_Int elem_bytes, int64_t n, HYPRE_Int reps, HYPRE_Real *avg_ms);
HYPRE_Int hypreve_DeviceSynchronize(void);
const char *hypreve_BuildInfo(void);
const char *hypreve_LastErrorMessage(void);

#ifdef __cplusplus
}
#endif
#endif /* HYPREVE_H */
