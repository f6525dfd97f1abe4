// Distributed BoomerAMG setup: every rank builds the levels of its own rows.
//
// hypre's setup is distributed (ParCSR, MPI); this one reproduces the
// single-process hierarchy of setup.cpp exactly -- same C points, same P and
// coarse operators, entry for entry and bit for bit -- while each rank only
// holds its rows plus a ghost layer of neighbour rows:
//   * strength: row-local;
//   * PMIS (coarsen_type 8): the measure counts come from every rank's S rows,
//     the random part is the reference's sequential stream evaluated at the
//     global row index, and each independent-set pass exchanges the measures,
//     the demotions and the C/F state of ghost points (the pass is
//     order-free, so the outcome equals the one-process pass);
//   * ext+i: rows computed by extpi_core over [owned | ghost] points, with the
//     A and S rows of the strong neighbours fetched from their owners;
//   * R = P^T: P entries sent to the owner of their coarse column, sorted by
//     fine row (the transpose's order);
//   * RAP: rap_core over the fine rows R touches and their A and P rows;
//   * l1 norms, the coarsest dense operator (gathered everywhere), statistics.
// The result is this rank's RankHierarchy, the same object the rank-0 gather
// path produces with partition_hierarchy (partition.hpp).  Other coarsening /
// interpolation types return an error and the caller takes the gather path.
#pragma once
#include <string>

#include "hostcomm.hpp"
#include "hve_host.hpp"
#include "partition.hpp"

namespace hve {

// Whether amg_setup_dist supports these parameters.
bool dist_setup_supported(const AMGParams& prm, std::string* why = nullptr);

// A0: this rank's rows (contiguous, starting at global row first_row, in rank
// order), global column indices, diagonal first.  Returns 0 on success.
int amg_setup_dist(const CSR& A0, int first_row, const AMGParams& prm, HostComm& comm, RankHierarchy& out,
                   std::string* log = nullptr);

// CPU self-check: the distributed setup on `size` host threads against
// partition_hierarchy of the one-process setup, compared as serialized bytes.
int dist_setup_self_check(const CSR& A, const AMGParams& prm, int size, std::string& msg);

}  // namespace hve
