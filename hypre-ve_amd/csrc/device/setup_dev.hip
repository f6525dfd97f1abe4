// Device setup kernels: the heavy row loops of the BoomerAMG setup
// (ext+i interpolation, its truncation, R = P^T and the Galerkin product RAP)
// run on the GPU, byte for byte what the host functions of host/setup.cpp
// produce.
//
// Each row of ext+i and RAP is an ordered first-touch list with sums formed in
// a fixed order, so one lane restates the host row function verbatim: one row
// per wavefront, lane 0 does the row's work, and the per-row marker map (the
// reference's P_marker / A_marker arrays, host RowMap) is an open-addressing
// table in the wave's LDS with generation stamps (no clearing between rows).
// Thousands of rows run at once, each an L1/LDS-latency chain, which is what
// makes the device versions fast: the host's rows are cache-miss chains into
// multi-GB arrays.  A row whose table would overflow its LDS capacity is
// flagged and finished by the host's own row function (setup.cpp), so every
// row is exact either way.  Truncation (par_csr_matrix.c:2671) runs one row
// per lane with the row in private memory; the quicksort partitions of
// qsort2_abs (hypre_qsort.c:367) are replayed from an explicit stack: the
// subranges are disjoint, so the order they are processed in does not change
// the result.  R = P^T is a stable radix sort of P's entries by column
// (rows stay ascending inside a column, as in the counting-sort transpose).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../host/setup_dev.hpp"
#include "kernels.h"

namespace hve {

namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("device setup: HIP error '") + hipGetErrorString(e) + "' in " + what);
}
#define SDV(x) ck((x), #x)

template <typename T>
struct DBuf {
  T* p = nullptr;
  size_t n = 0;
  DBuf() = default;
  explicit DBuf(size_t m) { alloc(m); }
  void alloc(size_t m) {
    free();
    n = m;
    SDV(hipMalloc((void**)&p, std::max<size_t>(1, m) * sizeof(T)));
  }
  template <typename Al>
  void up(const std::vector<T, Al>& h) {
    alloc(h.size());
    if (!h.empty()) SDV(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
  }
  template <typename Al>
  void down(std::vector<T, Al>& h, size_t m) const {
    h.resize(m);
    if (m) SDV(hipMemcpy(h.data(), p, m * sizeof(T), hipMemcpyDeviceToHost));
  }
  void free() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  ~DBuf() { free(); }
  DBuf(const DBuf&) = delete;
  DBuf& operator=(const DBuf&) = delete;
};

struct DCsr {
  const int* i;
  const int* j;
  const double* a;
  int n;
};

struct DevCSR {
  DBuf<int> i, j;
  DBuf<double> a;
  int n = 0, ncols = 0;
  void up(const CSR& h) {
    n = h.nrows;
    ncols = h.ncols;
    i.up(h.i);
    j.up(h.j);
    a.up(h.a);
  }
  DCsr view() const { return DCsr{i.p, j.p, a.p, n}; }
};

long long g_host_rows = 0;

// Device copies of one setup level's matrices (A, S, P), so that strength /
// PMIS, ext+i and RAP upload each once: keyed by the host arrays' addresses
// and sizes, and emptied by amg_setup at the start of every level (within a
// level the host A, S and P are not modified between the device calls).
struct SetupCache {
  const void *aj = nullptr, *aa = nullptr;
  int64_t annz = -1;
  int an = -1;
  DevCSR A;
  const void* sj = nullptr;
  int64_t snnz = -1;
  int sn = -1;
  DBuf<int> Si, Sj;
  const void *pj = nullptr, *pa = nullptr;
  int64_t pnnz = -1;
  int pn = -1;
  DevCSR P;
  void clear() {
    A.i.free(); A.j.free(); A.a.free();
    Si.free(); Sj.free();
    P.i.free(); P.j.free(); P.a.free();
    aj = aa = sj = pj = pa = nullptr;
    annz = snnz = pnnz = -1;
    an = sn = pn = -1;
  }
  const DevCSR& matA(const CSR& h) {
    if (!(aj == (const void*)h.j.data() && aa == (const void*)h.a.data() && annz == (int64_t)h.nnz() && an == h.nrows)) {
      A.up(h);
      aj = h.j.data(); aa = h.a.data(); annz = h.nnz(); an = h.nrows;
    }
    return A;
  }
  DCsr patS(const Pattern& h) {
    if (!(sj == (const void*)h.j.data() && snnz == (int64_t)h.j.size() && sn == h.n)) {
      Si.up(h.i);
      Sj.up(h.j);
      sj = h.j.data(); snnz = (int64_t)h.j.size(); sn = h.n;
    }
    return DCsr{Si.p, Sj.p, nullptr, h.n};
  }
  void keepS(const Pattern& h) { sj = h.j.data(); snnz = (int64_t)h.j.size(); sn = h.n; }
  const DevCSR& matP(const CSR& h) {
    if (!(pj == (const void*)h.j.data() && pa == (const void*)h.a.data() && pnnz == (int64_t)h.nnz() && pn == h.nrows)) {
      P.up(h);
      pj = h.j.data(); pa = h.a.data(); pnnz = h.nnz(); pn = h.nrows;
    }
    return P;
  }
  void keepP(const CSR& h) { pj = h.j.data(); pa = h.a.data(); pnnz = h.nnz(); pn = h.nrows; P.n = h.nrows; P.ncols = h.ncols; }
};
// never destroyed: its buffers must not be freed after the HIP runtime is gone
SetupCache& cache() {
  static SetupCache* c = new SetupCache();
  return *c;
}
template <typename T>
void take(DBuf<T>& dst, DBuf<T>& src) {
  dst.free();
  dst.p = src.p;
  dst.n = src.n;
  src.p = nullptr;
  src.n = 0;
}

// HVE_SETUP_T: stage times of the device setup on stderr
struct STimer {
  bool on = getenv("HVE_SETUP_T") != nullptr;
  double t = now();
  static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  void lap(const char* what) {
    if (!on) return;
    (void)hipDeviceSynchronize();
    const double n = now();
    fprintf(stderr, "[dsetup] %-28s %.3fs\n", what, n - t);
    t = n;
  }
};

// Open-addressing map in LDS, one per wavefront, used by lane 0 only.
struct LMap {
  int* key;
  int* val;
  int* gen;
  unsigned mask;
  int shift;
  int cur;
  int count;
  int limit;  // at most cap/2 keys: beyond that the row overflows
  __device__ void init(int* base, int cap, int lg) {
    key = base;
    val = base + cap;
    gen = base + 2 * cap;
    mask = (unsigned)cap - 1;
    shift = 32 - lg;
    cur = 0;
    limit = cap / 2;
  }
  __device__ void begin() {
    ++cur;
    count = 0;
  }
  // slot of k; inserted with v0 when absent (fresh); nullptr on overflow
  __device__ int* find_or_insert(int k, int v0, bool& fresh) {
    unsigned h = ((unsigned)k * 2654435761u) >> shift;
    for (;; h = (h + 1) & mask) {
      if (gen[h] != cur) {
        if (count >= limit) return nullptr;
        ++count;
        gen[h] = cur;
        key[h] = k;
        val[h] = v0;
        fresh = true;
        return &val[h];
      }
      if (key[h] == k) {
        fresh = false;
        return &val[h];
      }
    }
  }
  __device__ int get(int k, int dflt) const {
    unsigned h = ((unsigned)k * 2654435761u) >> shift;
    for (;; h = (h + 1) & mask) {
      if (gen[h] != cur) return dflt;
      if (key[h] == k) return val[h];
    }
  }
};

__device__ __forceinline__ void lds_zero(int* p, int n) {
  for (int t = threadIdx.x; t < n; t += blockDim.x) p[t] = 0;
  __syncthreads();
}

constexpr int kSF = -3;  // SF_PT

// ---------------------------------------------------------------------------
// Ext+i rows (setup.cpp extpi_row_count / extpi_row_fill, par_lr_interp.c:1041).
// COUNT: rowcnt[i] = |C-hat_i| (-1: overflow).  FILL: P.j / P.a of rows
// with rowcnt >= 0, from Pi[i] on.
// LDS: map (3 x cap ints) + the row's values (cap/2 doubles).
// ---------------------------------------------------------------------------
template <bool FILL>
__global__ void __launch_bounds__(64) k_extpi(DCsr A, DCsr S, const int* __restrict__ cf,
                                              const int* __restrict__ f2c, int n, int cap, int lg,
                                              int* __restrict__ rowcnt, const int* __restrict__ Pi,
                                              int* __restrict__ Pj, double* __restrict__ Pa) {
  extern __shared__ int lds[];
  lds_zero(lds + 2 * cap, cap);  // generation stamps
  if (threadIdx.x != 0) return;
  LMap M;
  M.init(lds, cap, lg);
  double* pa = reinterpret_cast<double*>(lds + 3 * cap);  // cap/2 doubles (8-aligned: cap is a power of 2)
  constexpr int kNone = -1, kStrongF = -2;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int ci = cf[i];
    if (!FILL) {
      int cnt = 0;
      if (ci >= 0) {
        cnt = 1;
      } else if (ci != kSF) {
        // the same insertions as the fill pass (strong F neighbours too), so a
        // row that fits here fits there
        M.begin();
        bool fresh, ovf = false;
        for (int jj = S.i[i]; jj < S.i[i + 1] && !ovf; ++jj) {
          const int i1 = S.j[jj];
          const int c1 = cf[i1];
          if (c1 >= 0) {
            if (!M.find_or_insert(i1, 0, fresh)) ovf = true;
            else cnt += fresh;
          } else if (c1 != kSF) {
            if (!M.find_or_insert(i1, kStrongF, fresh)) { ovf = true; break; }
            for (int kk = S.i[i1]; kk < S.i[i1 + 1]; ++kk) {
              const int k1 = S.j[kk];
              if (cf[k1] >= 0) {
                if (!M.find_or_insert(k1, 0, fresh)) { ovf = true; break; }
                cnt += fresh;
              }
            }
          }
        }
        if (ovf) cnt = -1;
      }
      rowcnt[i] = cnt;
      continue;
    }
    if (rowcnt[i] < 0) continue;  // finished on the host
    const int jb = Pi[i];
    if (ci >= 0) {
      Pj[jb] = f2c[i];
      Pa[jb] = 1.0;
      continue;
    }
    if (ci == kSF) continue;
    M.begin();
    int jc = 0;  // slot relative to jb
    bool fresh;
    for (int jj = S.i[i]; jj < S.i[i + 1]; ++jj) {
      const int i1 = S.j[jj];
      const int c1 = cf[i1];
      if (c1 >= 0) {
        M.find_or_insert(i1, jc, fresh);  // fits: the count pass saw the same keys
        if (fresh) { Pj[jb + jc] = f2c[i1]; pa[jc] = 0.0; jc++; }
      } else if (c1 != kSF) {
        *M.find_or_insert(i1, kStrongF, fresh) = kStrongF;
        for (int kk = S.i[i1]; kk < S.i[i1 + 1]; ++kk) {
          const int k1 = S.j[kk];
          if (cf[k1] >= 0) {
            M.find_or_insert(k1, jc, fresh);
            if (fresh) { Pj[jb + jc] = f2c[k1]; pa[jc] = 0.0; jc++; }
          }
        }
      }
    }
    const int jend = jc;
    double diagonal = A.a[A.i[i]];
    for (int jj = A.i[i] + 1; jj < A.i[i + 1]; ++jj) {
      const int i1 = A.j[jj];
      const int m1 = M.get(i1, kNone);
      if (m1 >= 0) {
        pa[m1] += A.a[jj];
      } else if (m1 == kStrongF) {
        double sum = 0.0;
        int sgn = 1;
        if (A.a[A.i[i1]] < 0) sgn = -1;
        for (int jj1 = A.i[i1] + 1; jj1 < A.i[i1 + 1]; ++jj1) {
          const int i2 = A.j[jj1];
          if ((M.get(i2, kNone) >= 0 || i2 == i) && (sgn * A.a[jj1]) < 0) sum += A.a[jj1];
        }
        if (sum != 0) {
          const double distribute = A.a[jj] / sum;
          for (int jj1 = A.i[i1] + 1; jj1 < A.i[i1 + 1]; ++jj1) {
            const int i2 = A.j[jj1];
            const int m2 = M.get(i2, kNone);
            if (m2 >= 0 && (sgn * A.a[jj1]) < 0) pa[m2] += distribute * A.a[jj1];
            if (i2 == i && (sgn * A.a[jj1]) < 0) diagonal += distribute * A.a[jj1];
          }
        } else {
          diagonal += A.a[jj];
        }
      } else if (cf[i1] != kSF) {
        diagonal += A.a[jj];
      }
    }
    if (diagonal) {
      for (int k = 0; k < jend; ++k) pa[k] /= -diagonal;
    }
    for (int k = 0; k < jend; ++k) Pa[jb + k] = pa[k];
  }
}

// ---------------------------------------------------------------------------
// Wave-parallel count passes.  A row's count is the number of distinct keys
// its candidates insert, which does not depend on the insertion order, so the
// 64 lanes insert at once into an LDS set of (generation, key) words claimed
// by 64-bit compare-and-swap.  A row overflows (-1: the host finishes it)
// exactly when it has more than cap/2 distinct keys, as in the one-lane
// passes, so the fill passes see the same rows.
// ---------------------------------------------------------------------------
struct LSet {
  unsigned long long* t;
  unsigned mask;
  int shift;
  unsigned cap;
  __device__ void init(unsigned long long* base, int c, int lg) {
    t = base;
    cap = (unsigned)c;
    mask = (unsigned)c - 1;
    shift = 32 - lg;
  }
  // 1: inserted (fresh), 0: present, -1: no free slot found (the row overflows)
  __device__ int insert(int k, unsigned cur) const {
    unsigned h = ((unsigned)k * 2654435761u) >> shift;
    const unsigned long long want = ((unsigned long long)cur << 32) | (unsigned)k;
    for (unsigned probes = 0; probes < cap;) {
      const unsigned long long w = __hip_atomic_load(&t[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      if ((unsigned)(w >> 32) == cur) {
        if ((unsigned)w == (unsigned)k) return 0;
        h = (h + 1) & mask;
        ++probes;
        continue;
      }
      unsigned long long exp = w;
      if (__hip_atomic_compare_exchange_strong(&t[h], &exp, want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WAVEFRONT))
        return 1;
      // another lane claimed the slot: look at it again
    }
    return -1;
  }
};

__device__ __forceinline__ int wave_sum(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ext+i count (k_extpi<false>): |C-hat_i|, strong F neighbours taking table
// slots as in the fill pass.  LDS: cap 64-bit words.
// rowkeys (optional): the row's table keys (C-hat plus strong F neighbours; 0
// for C and SF rows), which size the fill pass's table (dev_extpi_interp)
__global__ void __launch_bounds__(64) k_extpi_count_w(DCsr S, const int* __restrict__ cf, int n, int cap, int lg,
                                                      int* __restrict__ rowcnt, int* __restrict__ rowkeys) {
  extern __shared__ unsigned long long lds64[];
  for (int t = threadIdx.x; t < cap; t += 64) lds64[t] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x;
  LSet M;
  M.init(lds64, cap, lg);
  const int limit = cap / 2;
  unsigned cur = 0;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int ci = cf[i];
    if (ci >= 0 || ci == kSF) {
      if (lane == 0) {
        rowcnt[i] = ci >= 0 ? 1 : 0;
        if (rowkeys) rowkeys[i] = 0;
      }
      continue;
    }
    ++cur;
    int cntc = 0, keys = 0, bad = 0;
    for (int jj = S.i[i] + lane; jj < S.i[i + 1] && !bad; jj += 64) {
      const int i1 = S.j[jj];
      const int c1 = cf[i1];
      if (c1 >= 0) {
        const int r = M.insert(i1, cur);
        if (r < 0) bad = 1;
        cntc += r > 0;
        keys += r > 0;
      } else if (c1 != kSF) {
        const int r = M.insert(i1, cur);
        if (r < 0) bad = 1;
        keys += r > 0;
        for (int kk = S.i[i1]; kk < S.i[i1 + 1] && !bad; ++kk) {
          const int k1 = S.j[kk];
          if (cf[k1] >= 0) {
            const int r2 = M.insert(k1, cur);
            if (r2 < 0) bad = 1;
            cntc += r2 > 0;
            keys += r2 > 0;
          }
        }
      }
    }
    const int tk = wave_sum(keys), tc = wave_sum(cntc), tb = wave_sum(bad);
    if (lane == 0) {
      rowcnt[i] = (tb || tk > limit) ? -1 : tc;
      if (rowkeys) rowkeys[i] = tk;
    }
  }
}

// Galerkin count (k_rap<false>): distinct columns of C row q (q itself
// first).  LDS: cap1 + cap2 64-bit words and the RA list (cap1 / 2 ints).
__global__ void __launch_bounds__(64) k_rap_count_w(DCsr R, DCsr A, DCsr P, int cap1, int lg1, int cap2, int lg2,
                                                    int* __restrict__ rowlen, int* __restrict__ rownra) {
  extern __shared__ unsigned long long lds64[];
  for (int t = threadIdx.x; t < cap1 + cap2; t += 64) lds64[t] = 0ull;
  int* ra = reinterpret_cast<int*>(lds64 + cap1 + cap2);
  __shared__ int nra_s;
  __syncthreads();
  const int lane = threadIdx.x;
  LSet M1, M2;
  M1.init(lds64, cap1, lg1);
  M2.init(lds64 + cap1, cap2, lg2);
  const int lim1 = cap1 / 2, lim2 = cap2 / 2;
  unsigned cur = 0;
  for (int q = blockIdx.x; q < R.n; q += gridDim.x) {
    ++cur;
    if (lane == 0) nra_s = 0;
    __syncthreads();
    int bad = 0;
    for (int jj1 = R.i[q] + lane; jj1 < R.i[q + 1] && !bad; jj1 += 64) {
      const int i1 = R.j[jj1];
      for (int jj2 = A.i[i1]; jj2 < A.i[i1 + 1]; ++jj2) {
        const int i2 = A.j[jj2];
        const int r = M1.insert(i2, cur);
        if (r < 0) { bad = 1; break; }
        if (r > 0) {
          const int at = atomicAdd(&nra_s, 1);
          if (at < lim1) ra[at] = i2;
        }
      }
    }
    __syncthreads();
    const int nra = nra_s;
    int keys = 0;
    bad = wave_sum(bad);
    if (!bad && nra <= lim1) {
      if (lane == 0) keys += M2.insert(q, cur) > 0;
      __syncthreads();
      for (int t = lane; t < nra && !bad; t += 64) {
        const int i1 = ra[t];
        for (int jj2 = P.i[i1]; jj2 < P.i[i1 + 1]; ++jj2) {
          const int r = M2.insert(P.j[jj2], cur);
          if (r < 0) { bad = 1; break; }
          keys += r > 0;
        }
      }
      bad = wave_sum(bad);
      keys = wave_sum(keys);
    } else {
      bad = 1;
    }
    if (lane == 0) {
      rowlen[q] = (bad || keys > lim2) ? -1 : keys;
      if (rownra) rownra[q] = nra;
    }
    __syncthreads();
  }
}

// LDS writes of one lane visible to the wave's other lanes
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Fill pass with the wave's 64 lanes sharing the strong-F distribution loops
// (par_lr_interp.c's "sum" and "distribute" loops over A's row i1): lane 0
// builds C-hat in first-touch order as above; then for each entry of A's row i
// (in order, every lane in step) the lanes look up a chunk of row i1's entries
// in the LDS map at once.  The sum is still added up by lane 0 in entry order
// from the staged contributions, each distributed entry updates its own C-hat
// slot (a row holds a column once, so no two lanes meet), and the diagonal's
// single contribution of row i1 is added by every lane's copy of the diagonal
// in the same place as on the host.  Same operations, same order.
// keys / (kmin, kmax]: only the rows whose table keys fall in the range (a
// launch with a small table for the many short rows, another for the rest)
__global__ void __launch_bounds__(64) k_extpi_fill_w(DCsr A, DCsr S, const int* __restrict__ cf,
                                                     const int* __restrict__ f2c, int n, int cap, int lg,
                                                     const int* __restrict__ rowcnt, const int* __restrict__ Pi,
                                                     int* __restrict__ Pj, double* __restrict__ Pa,
                                                     const int* __restrict__ keys, int kmin, int kmax) {
  extern __shared__ int lds[];
  lds_zero(lds + 2 * cap, cap);  // generation stamps
  const int lane = threadIdx.x;
  LMap M;
  M.init(lds, cap, lg);
  double* pa = reinterpret_cast<double*>(lds + 3 * cap);  // cap/2 doubles
  double* cv = pa + cap / 2;                               // 64 staged contributions
  int* cfg = reinterpret_cast<int*>(cv + 64);              // 64 flags
  constexpr int kNone = -1, kStrongF = -2;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    if (rowcnt[i] < 0) continue;  // finished on the host
    if (keys && (keys[i] <= kmin || keys[i] > kmax)) continue;  // the other launch's row
    const int ci = cf[i];
    const int jb = Pi[i];
    if (ci >= 0) {
      if (lane == 0) {
        Pj[jb] = f2c[i];
        Pa[jb] = 1.0;
      }
      continue;
    }
    if (ci == kSF) continue;
    M.begin();  // every lane: the generation stamps stay in step
    int jend = 0;
    if (lane == 0) {
      int jc = 0;
      bool fresh;
      for (int jj = S.i[i]; jj < S.i[i + 1]; ++jj) {
        const int i1 = S.j[jj];
        const int c1 = cf[i1];
        if (c1 >= 0) {
          M.find_or_insert(i1, jc, fresh);
          if (fresh) { Pj[jb + jc] = f2c[i1]; pa[jc] = 0.0; jc++; }
        } else if (c1 != kSF) {
          *M.find_or_insert(i1, kStrongF, fresh) = kStrongF;
          for (int kk = S.i[i1]; kk < S.i[i1 + 1]; ++kk) {
            const int k1 = S.j[kk];
            if (cf[k1] >= 0) {
              M.find_or_insert(k1, jc, fresh);
              if (fresh) { Pj[jb + jc] = f2c[k1]; pa[jc] = 0.0; jc++; }
            }
          }
        }
      }
      jend = jc;
    }
    jend = __shfl(jend, 0, 64);
    wsync();
    double diagonal = A.a[A.i[i]];
    for (int jj = A.i[i] + 1; jj < A.i[i + 1]; ++jj) {
      const int i1 = A.j[jj];
      const double aij = A.a[jj];
      const int m1 = M.get(i1, kNone);
      if (m1 >= 0) {
        if (lane == 0) pa[m1] += aij;
        wsync();
      } else if (m1 == kStrongF) {
        const int b1 = A.i[i1] + 1, e1 = A.i[i1 + 1];
        const int sgn = (A.a[A.i[i1]] < 0) ? -1 : 1;
        double sum = 0.0;
        for (int c0 = b1; c0 < e1; c0 += 64) {
          const int jj1 = c0 + lane;
          double v = 0.0;
          int take = 0;
          if (jj1 < e1) {
            const int i2 = A.j[jj1];
            v = A.a[jj1];
            take = ((M.get(i2, kNone) >= 0 || i2 == i) && (sgn * v) < 0) ? 1 : 0;
          }
          cv[lane] = v;
          cfg[lane] = take;
          wsync();
          if (lane == 0) {
            const int cnt = min(64, e1 - c0);
            for (int q = 0; q < cnt; ++q)
              if (cfg[q]) sum += cv[q];
          }
          wsync();
        }
        sum = __shfl(sum, 0, 64);
        if (sum != 0) {
          const double distribute = aij / sum;
          double dadd = 0.0;
          int dhas = 0;
          for (int c0 = b1; c0 < e1; c0 += 64) {
            const int jj1 = c0 + lane;
            if (jj1 < e1) {
              const int i2 = A.j[jj1];
              const double a2 = A.a[jj1];
              const int m2 = M.get(i2, kNone);
              if (m2 >= 0 && (sgn * a2) < 0) pa[m2] += distribute * a2;
              if (i2 == i && (sgn * a2) < 0) {
                dadd = distribute * a2;
                dhas = 1;
              }
            }
          }
          const unsigned long long bl = __ballot(dhas);
          if (bl) diagonal += __shfl(dadd, __ffsll((long long)bl) - 1, 64);
          wsync();
        } else {
          diagonal += aij;
        }
      } else if (cf[i1] != kSF) {
        diagonal += aij;
      }
    }
    for (int k = lane; k < jend; k += 64) {
      double v = pa[k];
      if (diagonal) v /= -diagonal;
      Pa[jb + k] = v;
    }
    wsync();
  }
}

// ---------------------------------------------------------------------------
// Truncation of one row per lane (setup.cpp truncate_row): in place inside
// the row's slots, newlen[r] = kept entries (-1: row longer than kTrMax,
// finished on the host).
// ---------------------------------------------------------------------------
constexpr int kTrMax = 64;
__global__ void __launch_bounds__(256) k_truncate(int n, const int* __restrict__ Pi, int* __restrict__ Pj,
                                                  double* __restrict__ Pa, double tol, int max_elmts,
                                                  int* __restrict__ newlen) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const int b = Pi[r], e = Pi[r + 1];
  int len = e - b;
  if (len > kTrMax) {
    newlen[r] = -1;
    return;
  }
  int rj[kTrMax];
  double ra[kTrMax];
  for (int k = 0; k < len; ++k) {
    rj[k] = Pj[b + k];
    ra[k] = Pa[b + k];
  }
  if (tol > 0) {
    double row_nrm = 0;
    for (int k = 0; k < len; ++k) row_nrm = (row_nrm < fabs(ra[k])) ? fabs(ra[k]) : row_nrm;
    const double drop = tol * row_nrm;
    double row_sum = 0, scale = 0;
    int o = 0;
    for (int k = 0; k < len; ++k) {
      row_sum += ra[k];
      if (!(fabs(ra[k]) < drop)) { scale += ra[k]; rj[o] = rj[k]; ra[o] = ra[k]; ++o; }
    }
    len = o;
    if (scale != 0. && scale != row_sum) {
      scale = row_sum / scale;
      for (int k = 0; k < len; ++k) ra[k] *= scale;
    }
  }
  if (max_elmts > 0 && len > max_elmts) {
    double row_sum = 0;
    for (int k = 0; k < len; ++k) row_sum += ra[k];
    // qsort2_abs (descending |w|), its partitions replayed from a stack
    int stk[4 * kTrMax + 4];
    int sp = 0;
    stk[sp++] = 0;
    stk[sp++] = len - 1;
    while (sp > 0) {
      const int right = stk[--sp];
      const int left = stk[--sp];
      if (left >= right) continue;
      {
        const int m = (left + right) / 2;
        const int tv = rj[left]; rj[left] = rj[m]; rj[m] = tv;
        const double tw = ra[left]; ra[left] = ra[m]; ra[m] = tw;
      }
      int last = left;
      for (int k = left + 1; k <= right; ++k)
        if (fabs(ra[k]) > fabs(ra[left])) {
          ++last;
          const int tv = rj[last]; rj[last] = rj[k]; rj[k] = tv;
          const double tw = ra[last]; ra[last] = ra[k]; ra[k] = tw;
        }
      {
        const int tv = rj[left]; rj[left] = rj[last]; rj[last] = tv;
        const double tw = ra[left]; ra[left] = ra[last]; ra[last] = tw;
      }
      stk[sp++] = left;
      stk[sp++] = last - 1;
      stk[sp++] = last + 1;
      stk[sp++] = right;
    }
    double scale = 0;
    for (int k = 0; k < max_elmts; ++k) scale += ra[k];
    len = max_elmts;
    if (scale != 0. && scale != row_sum) {
      scale = row_sum / scale;
      for (int k = 0; k < len; ++k) ra[k] *= scale;
    }
  }
  for (int k = 0; k < len; ++k) {
    Pj[b + k] = rj[k];
    Pa[b + k] = ra[k];
  }
  newlen[r] = len;
}

// compacted copy of the kept entries: row r's newlen[r] first slots
__global__ void __launch_bounds__(256) k_compact(int n, const int* __restrict__ Pi, const int* __restrict__ Pj,
                                                 const double* __restrict__ Pa, const int* __restrict__ Ni,
                                                 int* __restrict__ Nj, double* __restrict__ Na) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const int b = Pi[r], o = Ni[r], len = Ni[r + 1] - Ni[r];
  for (int k = 0; k < len; ++k) {
    Nj[o + k] = Pj[b + k];
    Na[o + k] = Pa[b + k];
  }
}

// ---------------------------------------------------------------------------
// Transpose helpers: row of every entry, column counts, gather of values.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_entry_rows(int n, const int* __restrict__ Pi, int* __restrict__ rowof) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  for (int k = Pi[r]; k < Pi[r + 1]; ++k) rowof[k] = r;
}
__global__ void __launch_bounds__(256) k_iota(int64_t n, int* __restrict__ v) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < n) v[k] = (int)k;
}
__global__ void __launch_bounds__(256) k_col_count(int64_t nnz, const int* __restrict__ Pj, int* __restrict__ cnt) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k < nnz) atomicAdd(&cnt[Pj[k]], 1);
}
__global__ void __launch_bounds__(256) k_transpose_fill(int64_t nnz, const int* __restrict__ perm,
                                                        const int* __restrict__ rowof, const double* __restrict__ Pa,
                                                        int* __restrict__ Rj, double* __restrict__ Ra) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= nnz) return;
  const int e = perm[k];
  Rj[k] = rowof[e];
  Ra[k] = Pa[e];
}

// ---------------------------------------------------------------------------
// Galerkin rows (setup.cpp rap_row, par_rap.c:27): C row q from R row q,
// the RA row (first touch over A's columns) and then RA * P (first touch over
// P's columns, the diagonal ic = q first).  COUNT: rowlen[q] (-1: overflow);
// FILL: C.j / C.a from Ci[q].  LDS: map1 (3 x cap1) + RA list (cap1/2 ints +
// doubles) + map2 (3 x cap2) + the row's values (cap2/2 doubles).
// ---------------------------------------------------------------------------
template <bool FILL>
// mode t > 0: only the rows of tier t, where tier 1 holds at most lim1a RA
// keys (rownra) and lim2a C keys (their length), tier 2 at most lim1b /
// lim2b, tier 3 the rest; mode 0: every row (dev_rap's table sizes)
__global__ void __launch_bounds__(64) k_rap(DCsr R, DCsr A, DCsr P, int cap1, int lg1, int cap2, int lg2,
                                            int* __restrict__ rowlen, const int* __restrict__ Ci,
                                            int* __restrict__ Cj, double* __restrict__ Ca,
                                            const int* __restrict__ rownra, int mode, int lim1a, int lim2a,
                                            int lim1b, int lim2b) {
  extern __shared__ int lds[];
  int* m1 = lds;
  int* m2 = m1 + 3 * cap1;
  lds_zero(m1 + 2 * cap1, cap1);
  lds_zero(m2 + 2 * cap2, cap2);
  if (threadIdx.x != 0) return;
  int* raj = m2 + 3 * cap2;                                        // cap1/2 ints
  double* raa = reinterpret_cast<double*>(raj + cap1 / 2);         // cap1/2 doubles
  double* ta = raa + cap1 / 2;                                     // cap2/2 doubles
  LMap M1, M2;
  M1.init(m1, cap1, lg1);
  M2.init(m2, cap2, lg2);
  for (int q = blockIdx.x; q < R.n; q += gridDim.x) {
    if (FILL && rowlen[q] < 0) continue;  // finished on the host
    if (FILL && mode) {
      const int na = rownra[q], nl = rowlen[q];
      const int tier = (na <= lim1a && nl <= lim2a) ? 1 : (na <= lim1b && nl <= lim2b) ? 2 : 3;
      if (tier != mode) continue;  // another launch's row
    }
    M1.begin();
    int nra = 0;
    bool fresh, ovf = false;
    for (int jj1 = R.i[q]; jj1 < R.i[q + 1] && !ovf; ++jj1) {
      const int i1 = R.j[jj1];
      const double r_entry = R.a[jj1];
      for (int jj2 = A.i[i1]; jj2 < A.i[i1 + 1]; ++jj2) {
        const int i2 = A.j[jj2];
        int* m = M1.find_or_insert(i2, nra, fresh);
        if (!m) { ovf = true; break; }
        if (fresh) {
          raj[nra] = i2;
          if (FILL) raa[nra] = r_entry * A.a[jj2];
          ++nra;
        } else if (FILL) {
          raa[*m] += r_entry * A.a[jj2];
        }
      }
    }
    int ntj = 0;
    if (!ovf) {
      M2.begin();
      M2.find_or_insert(q, 0, fresh);
      const int cb = FILL ? Ci[q] : 0;
      if (FILL) {
        Cj[cb] = q;
        ta[0] = 0.0;
      }
      ntj = 1;
      for (int k = 0; k < nra && !ovf; ++k) {
        const int i1 = raj[k];
        const double rap_ = FILL ? raa[k] : 0.0;
        for (int jj2 = P.i[i1]; jj2 < P.i[i1 + 1]; ++jj2) {
          const int i2 = P.j[jj2];
          int* m = M2.find_or_insert(i2, ntj, fresh);
          if (!m) { ovf = true; break; }
          if (fresh) {
            if (FILL) {
              Cj[cb + ntj] = i2;
              ta[ntj] = rap_ * P.a[jj2];
            }
            ++ntj;
          } else if (FILL) {
            ta[*m] += rap_ * P.a[jj2];
          }
        }
      }
      if (FILL)
        for (int k = 0; k < ntj; ++k) Ca[cb + k] = ta[k];
    }
    if (!FILL) rowlen[q] = ovf ? -1 : ntj;
  }
}

int lg2_ceil(int64_t v) {
  int lg = 4;
  while ((int64_t(1) << lg) < v) ++lg;
  return lg;
}

void exclusive_scan(const int* d_in, int* d_out, int n) {
  size_t tmp = 0;
  SDV(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, d_in, d_out, n));
  DBuf<char> t(tmp);
  SDV(hipcub::DeviceScan::ExclusiveSum(t.p, tmp, d_in, d_out, n));
}

// Row pointers from per-row counts (device), with the host copy.
void row_ptr(const DBuf<int>& cnt, int n, DBuf<int>& ptr, std::vector<int>& hptr) {
  ptr.alloc((size_t)n + 1);
  std::vector<int> hc;
  cnt.down(hc, n);
  hptr.assign((size_t)n + 1, 0);
  int64_t t = 0;
  for (int r = 0; r < n; ++r) {
    hptr[r] = (int)t;
    t += hc[r];
  }
  if (t > 0x7fffffffLL) throw std::runtime_error("device setup: more than 2^31 entries");
  hptr[n] = (int)t;
  SDV(hipMemcpy(ptr.p, hptr.data(), hptr.size() * sizeof(int), hipMemcpyHostToDevice));
}

int grid_rows(int n, int waves_per_cu) { return std::max(1, std::min(n, 256 * waves_per_cu)); }

// ---------------------------------------------------------------------------
// Strength of connection (setup.cpp create_strength, par_strength.c:80, one
// function): one row per thread, the row's scale and sum over its entries in
// stored order, the same comparisons.  FILL: the kept columns in order.
// ---------------------------------------------------------------------------
template <bool FILL>
__global__ void __launch_bounds__(256) k_strength(DCsr A, double thr, double max_row_sum, int* __restrict__ cnt,
                                                  const int* __restrict__ Si, int* __restrict__ Sj) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= A.n) return;
  const int b = A.i[r], e = A.i[r + 1];
  const double diag = A.a[b];
  double row_scale = 0.0, row_sum = diag;
  // std::max / std::min as on the host (the first argument on ties)
  if (diag < 0) {
    for (int k = b + 1; k < e; ++k) { const double v = A.a[k]; row_scale = row_scale < v ? v : row_scale; row_sum += v; }
  } else {
    for (int k = b + 1; k < e; ++k) { const double v = A.a[k]; row_scale = v < row_scale ? v : row_scale; row_sum += v; }
  }
  const bool weak = (fabs(row_sum) > fabs(diag) * max_row_sum) && (max_row_sum < 1.0);
  int c = 0, o = FILL ? Si[r] : 0;
  if (!weak) {
    for (int k = b + 1; k < e; ++k) {
      const double v = A.a[k];
      const bool keep = diag < 0 ? !(v <= thr * row_scale) : !(v >= thr * row_scale);
      if (keep) {
        if (FILL) Sj[o++] = A.j[k];
        ++c;
      }
    }
  }
  if (!FILL) cnt[r] = c;
}

// ---------------------------------------------------------------------------
// PMIS (setup.cpp coarsen_pmis, par_coarsen.c:2031, one process, CF_init 0 /
// 2: the one-process streams agree).  measure = column count of S + the
// row's hypre_Rand draw (seed 2747, draw r + 1: A^(r+1) seed mod M), then the
// host loop's passes as kernels over the rows still undecided (act), each
// pass order-free as on the host (the independent-set pass only writes 0).
// ---------------------------------------------------------------------------
constexpr uint64_t kDRandA = 16807, kDRandM = 2147483647;  // setup.cpp hypre_Rand (utilities/random.c)
__device__ uint64_t d_powmod(uint64_t b, uint64_t e, uint64_t m) {
  uint64_t r = 1;
  b %= m;
  while (e) {
    if (e & 1) r = (r * b) % m;
    b = (b * b) % m;
    e >>= 1;
  }
  return r;
}
__global__ void __launch_bounds__(256) k_pmis_init(int n, const int* __restrict__ Si, const int* __restrict__ mcount,
                                                   double* __restrict__ measure, int* __restrict__ cf,
                                                   unsigned char* __restrict__ act) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= n) return;
  const uint64_t s = (d_powmod(kDRandA, (uint64_t)r + 1, kDRandM) * 2747ull) % kDRandM;
  double m = (double)mcount[r];
  m += (double)s / (double)kDRandM;
  if (Si[r + 1] - Si[r] == 0) {
    cf[r] = -3;  // SF_PT (par_coarsen.c:2320-2326)
    m = 0;
    act[r] = 0;
  } else {
    cf[r] = 0;
    act[r] = 1;
  }
  measure[r] = m;
}
// pass 1: the initial independent set (measure > 1)
__global__ void __launch_bounds__(256) k_pmis_mark(int n, const unsigned char* __restrict__ act,
                                                   const double* __restrict__ measure, int* __restrict__ cf) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r < n && act[r] && measure[r] > 1) cf[r] = 1;
}
// pass 2: drop the smaller of two strongly connected candidates (writes 0 only)
__global__ void __launch_bounds__(256) k_pmis_drop(int n, const unsigned char* __restrict__ act, const int* __restrict__ Si,
                                                   const int* __restrict__ Sj, const double* __restrict__ measure,
                                                   int* __restrict__ cf) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n || !act[i]) return;
  const double mi = measure[i];
  if (!(mi > 1)) return;
  for (int k = Si[i]; k < Si[i + 1]; ++k) {
    const int j = Sj[k];
    const double mj = measure[j];
    if (mj > 1) {
      if (mi > mj) __hip_atomic_store(&cf[j], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if (mj > mi) __hip_atomic_store(&cf[i], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
// pass 3: C and F points (a marker > 0 stays, so the reads are order-free)
__global__ void __launch_bounds__(256) k_pmis_set(int n, const unsigned char* __restrict__ act, const int* __restrict__ Si,
                                                  const int* __restrict__ Sj, const double* __restrict__ measure,
                                                  int* __restrict__ cf) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n || !act[i]) return;
  int v = cf[i];
  if (measure[i] < 1) v = -1;  // F_PT
  if (v > 0) {
    v = 1;  // C_PT
  } else {
    for (int k = Si[i]; k < Si[i + 1]; ++k)
      if (__hip_atomic_load(&cf[Sj[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0) { v = -1; break; }
  }
  if (v != cf[i]) __hip_atomic_store(&cf[i], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// pass 4: decided rows leave the graph (measure 0); the rest are counted
__global__ void __launch_bounds__(256) k_pmis_next(int n, unsigned char* __restrict__ act, double* __restrict__ measure,
                                                   const int* __restrict__ cf, int* __restrict__ left) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  int still = 0;
  if (i < n && act[i]) {
    if (cf[i] != 0) {
      measure[i] = 0;
      act[i] = 0;
    } else {
      still = 1;
    }
  }
  const unsigned long long b = __ballot(still);
  if ((threadIdx.x & 63) == 0 && b) atomicAdd(left, __popcll(b));
}

}  // namespace

long long dev_setup_host_rows() { return g_host_rows; }

void dev_setup_cache_clear() { cache().clear(); }

void dev_strength_pmis(const CSR& A, double thr, double max_row_sum, Pattern& S, std::vector<int>& cf,
                       double* t_strength) {
  const int n = A.nrows;
  const auto t0 = STimer::now();
  STimer T;
  S.n = n;
  S.i.assign((size_t)n + 1, 0);
  S.j.clear();
  cf.assign(n, 0);
  if (n == 0) return;
  const dim3 g((n + 255) / 256), b(256);
  SetupCache& C = cache();
  DBuf<int>& Si = C.Si;
  DBuf<int>& Sj = C.Sj;
  {
    const DevCSR& dA = C.matA(A);  // kept for ext+i and RAP
    T.lap("strength: A upload");
    DBuf<int> cnt(n);
    hipLaunchKernelGGL((k_strength<false>), g, b, 0, 0, dA.view(), thr, max_row_sum, cnt.p, nullptr, nullptr);
    SDV(hipGetLastError());
    row_ptr(cnt, n, Si, S.i);
    T.lap("strength: count, row starts");
    Sj.alloc((size_t)S.i[n]);
    hipLaunchKernelGGL((k_strength<true>), g, b, 0, 0, dA.view(), thr, max_row_sum, nullptr, Si.p, Sj.p);
    SDV(hipGetLastError());
    T.lap("strength: fill");
    Sj.down(S.j, (size_t)S.i[n]);
    C.keepS(S);  // S stays on the device for ext+i
  }
  T.lap("strength: S download");
  if (t_strength) *t_strength = STimer::now() - t0;
  const int64_t nnzs = S.i[n];
  DBuf<int> mc(n), dcf(n), left(1);
  DBuf<double> meas(n);
  DBuf<unsigned char> act(n);
  SDV(hipMemset(mc.p, 0, sizeof(int) * (size_t)n));
  if (nnzs > 0)
    hipLaunchKernelGGL(k_col_count, dim3((unsigned)((nnzs + 255) / 256)), b, 0, 0, nnzs, Sj.p, mc.p);
  hipLaunchKernelGGL(k_pmis_init, g, b, 0, 0, n, Si.p, mc.p, meas.p, dcf.p, act.p);
  SDV(hipGetLastError());
  for (int iter = 0; iter < 1000; ++iter) {
    hipLaunchKernelGGL(k_pmis_mark, g, b, 0, 0, n, act.p, meas.p, dcf.p);
    hipLaunchKernelGGL(k_pmis_drop, g, b, 0, 0, n, act.p, Si.p, Sj.p, meas.p, dcf.p);
    hipLaunchKernelGGL(k_pmis_set, g, b, 0, 0, n, act.p, Si.p, Sj.p, meas.p, dcf.p);
    SDV(hipMemset(left.p, 0, sizeof(int)));
    hipLaunchKernelGGL(k_pmis_next, g, b, 0, 0, n, act.p, meas.p, dcf.p, left.p);
    SDV(hipGetLastError());
    int h = 0;
    SDV(hipMemcpy(&h, left.p, sizeof(int), hipMemcpyDeviceToHost));
    if (h == 0) break;
    if (iter == 999) throw std::runtime_error("device PMIS: no convergence after 1000 passes");
  }
  dcf.down(cf, n);
  T.lap("PMIS kernels");
}

void dev_extpi_interp(const CSR& A, const Pattern& S, const std::vector<int>& cf,
                      const std::vector<int>& fine_to_coarse, int ncoarse, double trunc_factor, int max_elmts,
                      CSR& P) {
  g_host_rows = 0;
  const int n = A.nrows;
  P.resize_rows(n, ncoarse);
  if (n == 0) return;
  STimer T;
  SetupCache& C = cache();
  const DevCSR& dA = C.matA(A);  // uploaded by the strength pass of this level, or now
  const DCsr dS = C.patS(S);
  DBuf<int> dcf, df2c;
  dcf.up(cf);
  df2c.up(fine_to_coarse);
  T.lap("extpi upload");
  // table capacity from the largest candidate count of a row (capped; rows
  // beyond it overflow to the host)
  const int64_t bmax = extpi_bound_max(S);
  // <= 2048 slots: 24 KiB + 8 KiB of values (knob 7 lowers the cap: tests of the host fallback)
  const int lg = std::min(lg2_ceil(2 * bmax + 2), knob(7) > 0 ? std::min(knob(7), 11) : 11);
  const int cap = 1 << lg;
  const size_t lds = (size_t)3 * cap * sizeof(int) + (size_t)(cap / 2) * sizeof(double);
  DBuf<int> cnt(n);
  const int grid = grid_rows(n, 32);
  // Rows with few candidates (the finest 7-point level: at most 43) run the
  // one-lane fill; the wave-shared one pays its synchronisation only on the
  // long Galerkin rows (512^3, level 0: 0.89 vs 4.3 s; level 1: 6.9 vs 1.6 s).
  const bool serial_fill = bmax <= 64;
  DBuf<int> keys(serial_fill ? 1 : (size_t)n);  // per-row table keys (the wave-shared fill's two launches)
  constexpr int pcount = 1;  // the wave-parallel count (one lane a row: level-1 ext+i count 1.7 s against 0.3 at 512^3)
  if (pcount)
    hipLaunchKernelGGL(k_extpi_count_w, dim3(grid), dim3(64), (size_t)cap * 8, 0, dS, dcf.p, n, cap, lg, cnt.p,
                       serial_fill ? nullptr : keys.p);
  else
    hipLaunchKernelGGL((k_extpi<false>), dim3(grid), dim3(64), lds, 0, dA.view(), dS, dcf.p, df2c.p, n, cap, lg, cnt.p,
                       nullptr, nullptr, nullptr);
  SDV(hipGetLastError());
  T.lap("extpi count kernel");
  // rows that overflowed: counted on the host
  std::vector<int> hc;
  cnt.down(hc, n);
  std::vector<int> ovf;
  for (int i = 0; i < n; ++i)
    if (hc[i] < 0) ovf.push_back(i);
  if (!ovf.empty()) extpi_count_rows(S, cf, ovf, hc);
  std::vector<int> hp((size_t)n + 1, 0);
  int64_t t = 0;
  for (int i = 0; i < n; ++i) {
    hp[i] = (int)t;
    t += hc[i];
  }
  if (t > 0x7fffffffLL) throw std::runtime_error("device setup: interpolation exceeds 2^31 entries");
  hp[n] = (int)t;
  DBuf<int> Pi, Pj((size_t)t);
  DBuf<double> Pa((size_t)t);
  Pi.up(hp);
  // the count buffer keeps -1 on overflow rows: the fill pass skips them.
  if (serial_fill) {
    hipLaunchKernelGGL((k_extpi<true>), dim3(grid), dim3(64), lds, 0, dA.view(), dS, dcf.p, df2c.p, n, cap, lg, cnt.p,
                       Pi.p, Pj.p, Pa.p);
  } else {
    // The wave-shared fill in tiers of table sizes: rows of at most 128
    // table keys with a 256-slot table (5 KiB of LDS a wave: 32 waves a CU),
    // at most 256 with 512 slots (9 KiB), the rest with the full table (up to
    // 33 KiB: 4 waves a CU), so the many shorter rows do not run at the long
    // rows' occupancy; the same entries in every tier.
    // (knob 19: the small table's log2 size, tests: every tier populated)
    const int lgs = knob(19) > 0 ? std::min(knob(19), 8) : 8;
    const size_t extra = 64 * (sizeof(double) + sizeof(int));
    auto ldsz = [](int c) { return (size_t)3 * c * sizeof(int) + (size_t)(c / 2) * sizeof(double); };
    if (cap > (1 << lgs)) {
      int lo = -1;
      for (int lt = lgs; lt <= lg; ++lt) {
        const int c = 1 << lt, hi = lt == lg ? 0x7fffffff : c / 2;
        hipLaunchKernelGGL(k_extpi_fill_w, dim3(grid), dim3(64), ldsz(c) + extra, 0, dA.view(), dS, dcf.p, df2c.p, n,
                           c, lt, cnt.p, Pi.p, Pj.p, Pa.p, keys.p, lo, hi);
        lo = hi;
        if (lt == lgs + 1 && lt < lg) lt = lg - 1;  // three tiers: small, twice small, full
      }
    } else {
      hipLaunchKernelGGL(k_extpi_fill_w, dim3(grid), dim3(64), lds + extra, 0, dA.view(), dS, dcf.p, df2c.p, n, cap, lg,
                         cnt.p, Pi.p, Pj.p, Pa.p, nullptr, 0, 0);
    }
  }
  SDV(hipGetLastError());
  T.lap("extpi fill kernel");
  const bool trunc = trunc_factor != 0.0 || max_elmts > 0;
  if (!trunc) {
    P.i = hp;
    Pj.down(P.j, (size_t)t);
    Pa.down(P.a, (size_t)t);
    if (!ovf.empty()) extpi_fill_rows(A, S, cf, fine_to_coarse, ovf, P);
    g_host_rows = (long long)ovf.size();
    return;
  }
  // overflow rows: filled on the host into the device arrays before truncation
  if (!ovf.empty()) {
    CSR part;
    part.resize_rows(n, ncoarse);
    part.i = hp;
    part.j.assign((size_t)t, 0);
    part.a.assign((size_t)t, 0.0);
    extpi_fill_rows(A, S, cf, fine_to_coarse, ovf, part);
    for (int i : ovf) {
      const int b = hp[i], len = hp[i + 1] - hp[i];
      if (len == 0) continue;
      SDV(hipMemcpy(Pj.p + b, part.j.data() + b, len * sizeof(int), hipMemcpyHostToDevice));
      SDV(hipMemcpy(Pa.p + b, part.a.data() + b, len * sizeof(double), hipMemcpyHostToDevice));
    }
  }
  DBuf<int> nl(n);
  hipLaunchKernelGGL(k_truncate, dim3((n + 255) / 256), dim3(256), 0, 0, n, Pi.p, Pj.p, Pa.p, trunc_factor, max_elmts,
                     nl.p);
  SDV(hipGetLastError());
  T.lap("truncate kernel");
  std::vector<int> hl;
  nl.down(hl, n);
  std::vector<int> longrows;
  for (int i = 0; i < n; ++i)
    if (hl[i] < 0) longrows.push_back(i);
  if (!longrows.empty()) {  // rows longer than the kernel's private arrays
    CSR part;
    part.resize_rows(n, ncoarse);
    part.i = hp;
    part.j.assign((size_t)t, 0);
    part.a.assign((size_t)t, 0.0);
    for (int i : longrows) {
      const int b = hp[i], len = hp[i + 1] - hp[i];
      SDV(hipMemcpy(part.j.data() + b, Pj.p + b, len * sizeof(int), hipMemcpyDeviceToHost));
      SDV(hipMemcpy(part.a.data() + b, Pa.p + b, len * sizeof(double), hipMemcpyDeviceToHost));
    }
    truncate_row_list(part, longrows, trunc_factor, max_elmts, hl);
    for (int i : longrows) {
      const int b = hp[i], len = hl[i];
      SDV(hipMemcpy(Pj.p + b, part.j.data() + b, len * sizeof(int), hipMemcpyHostToDevice));
      SDV(hipMemcpy(Pa.p + b, part.a.data() + b, len * sizeof(double), hipMemcpyHostToDevice));
    }
  }
  std::vector<int> ni((size_t)n + 1, 0);
  for (int i = 0; i < n; ++i) ni[i + 1] = ni[i] + hl[i];
  DBuf<int> Ni, Nj((size_t)ni[n]);
  DBuf<double> Na((size_t)ni[n]);
  Ni.up(ni);
  hipLaunchKernelGGL(k_compact, dim3((n + 255) / 256), dim3(256), 0, 0, n, Pi.p, Pj.p, Pa.p, Ni.p, Nj.p, Na.p);
  SDV(hipGetLastError());
  T.lap("truncate host part");
  P.i = ni;
  Nj.down(P.j, (size_t)ni[n]);
  Na.down(P.a, (size_t)ni[n]);
  T.lap("P download");
  g_host_rows = (long long)(ovf.size() + longrows.size());
  // the complete P (host-finished rows included) stays on the device for RAP
  take(C.P.i, Ni);
  take(C.P.j, Nj);
  take(C.P.a, Na);
  C.keepP(P);
}

void dev_rap(const CSR& P, const CSR& A, CSR& Rh, CSR& C) {
  g_host_rows = 0;
  const int nf = P.nrows, nc = P.ncols;
  const int64_t nnzp = P.nnz();
  STimer T;
  SetupCache& Cc = cache();
  const DevCSR& dP = Cc.matP(P);  // ext+i's device P, or uploaded now
  const DevCSR& dA = Cc.matA(A);
  T.lap("rap upload");
  // R = P^T: a stable radix sort of the entries by column keeps every
  // column's rows ascending (transpose's counting sort)
  DBuf<int> rowof((size_t)nnzp), perm_in((size_t)nnzp), keys_out((size_t)nnzp), perm((size_t)nnzp);
  hipLaunchKernelGGL(k_entry_rows, dim3((nf + 255) / 256), dim3(256), 0, 0, nf, dP.i.p, rowof.p);
  hipLaunchKernelGGL(k_iota, dim3((unsigned)((nnzp + 255) / 256)), dim3(256), 0, 0, nnzp, perm_in.p);
  SDV(hipGetLastError());
  {
    int bits = 1;
    while ((1LL << bits) < (int64_t)std::max(nc, 2)) ++bits;
    size_t tmp = 0;
    SDV(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, dP.j.p, keys_out.p, perm_in.p, perm.p, (int)nnzp, 0, bits));
    DBuf<char> t(tmp);
    SDV(hipcub::DeviceRadixSort::SortPairs(t.p, tmp, dP.j.p, keys_out.p, perm_in.p, perm.p, (int)nnzp, 0, bits));
  }
  perm_in.free();
  keys_out.free();
  DBuf<int> ccnt((size_t)nc + 1), Ri((size_t)nc + 1);
  SDV(hipMemset(ccnt.p, 0, ((size_t)nc + 1) * sizeof(int)));
  hipLaunchKernelGGL(k_col_count, dim3((unsigned)((nnzp + 255) / 256)), dim3(256), 0, 0, nnzp, dP.j.p, ccnt.p);
  exclusive_scan(ccnt.p, Ri.p, nc + 1);
  DBuf<int> Rj((size_t)nnzp);
  DBuf<double> Ra((size_t)nnzp);
  hipLaunchKernelGGL(k_transpose_fill, dim3((unsigned)((nnzp + 255) / 256)), dim3(256), 0, 0, nnzp, perm.p, rowof.p,
                     dP.a.p, Rj.p, Ra.p);
  SDV(hipGetLastError());
  perm.free();
  rowof.free();
  ccnt.free();
  Rh.resize_rows(nc, nf);
  Ri.down(Rh.i, (size_t)nc + 1);
  Rj.down(Rh.j, (size_t)nnzp);
  Ra.down(Rh.a, (size_t)nnzp);
  T.lap("transpose + R download");
  // table capacities from the largest products of a row (rows beyond: host)
  const int64_t b1 = rap_bound_max(Rh, A);
  int64_t pmax = 1;
  for (int r = 0; r < nf; ++r) pmax = std::max<int64_t>(pmax, P.i[r + 1] - P.i[r]);
  const int lgcap = knob(7) > 0 ? knob(7) : 10;
  const int lg1 = std::min(lg2_ceil(2 * b1 + 2), std::min(lgcap, 10));
  const int cap1 = 1 << lg1;
  const int lg2 = std::min(lg2_ceil(2 * (1 + (int64_t)(cap1 / 2) * pmax) + 2), std::min(lgcap, 9));
  const int cap2 = 1 << lg2;
  const size_t lds = (size_t)3 * (cap1 + cap2) * sizeof(int) + (size_t)(cap1 / 2) * (sizeof(int) + sizeof(double)) +
                     (size_t)(cap2 / 2) * sizeof(double);
  const DCsr dR{Ri.p, Rj.p, Ra.p, nc};
  DBuf<int> len((size_t)nc), nra((size_t)nc);  // C row lengths, RA keys a row
  const int grid = grid_rows(nc, 32);
  constexpr int pcount = 1;  // the wave-parallel count
  if (pcount)
    hipLaunchKernelGGL(k_rap_count_w, dim3(grid), dim3(64), (size_t)(cap1 + cap2) * 8 + (size_t)(cap1 / 2) * 4, 0, dR,
                       dA.view(), dP.view(), cap1, lg1, cap2, lg2, len.p, nra.p);
  else
    hipLaunchKernelGGL((k_rap<false>), dim3(grid), dim3(64), lds, 0, dR, dA.view(), dP.view(), cap1, lg1, cap2, lg2,
                       len.p, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, 0, 0);
  SDV(hipGetLastError());
  T.lap("rap count kernel");
  std::vector<int> hl;
  len.down(hl, nc);
  std::vector<int> ovf;
  for (int q = 0; q < nc; ++q)
    if (hl[q] < 0) ovf.push_back(q);
  std::vector<std::vector<int>> oj;
  std::vector<std::vector<double>> oa;
  rap_row_list(Rh, A, P, ovf, oj, oa);
  for (size_t k = 0; k < ovf.size(); ++k) hl[ovf[k]] = (int)oj[k].size();
  std::vector<int> ci((size_t)nc + 1, 0);
  for (int q = 0; q < nc; ++q) {
    if ((int64_t)ci[q] + hl[q] > 0x7fffffffLL) throw std::runtime_error("device setup: RAP exceeds 2^31 entries");
    ci[q + 1] = ci[q] + hl[q];
  }
  DBuf<int> Ci, Cj((size_t)ci[nc]);
  DBuf<double> Ca((size_t)ci[nc]);
  Ci.up(ci);
  // Tiers of table sizes: rows of at most 128 RA keys and 128 C keys with
  // 256-slot tables (8.5 KiB of LDS a wave), rows of at most 256 / 256 with
  // 512-slot ones (17 KiB), the rest with the full ones (26 KiB at 1024 /
  // 512), so the shorter rows run at a higher occupancy; the same entries in
  // every tier
  const int lgs = knob(19) > 0 ? std::min(knob(19), 8) : 8;  // knob 19 as in dev_extpi_interp
  auto ldsz = [](int c1, int c2) {
    return (size_t)3 * (c1 + c2) * sizeof(int) + (size_t)(c1 / 2) * (sizeof(int) + sizeof(double)) +
           (size_t)(c2 / 2) * sizeof(double);
  };
  const int ca1 = std::min(cap1, 1 << lgs), ca2 = std::min(cap2, 1 << lgs);
  const int cb1 = std::min(cap1, 2 << lgs), cb2 = std::min(cap2, 2 << lgs);
  if (cap1 > ca1 || cap2 > ca2) {
    const int la1 = std::min(lg1, lgs), la2 = std::min(lg2, lgs), lb1 = std::min(lg1, lgs + 1),
              lb2 = std::min(lg2, lgs + 1);
    const int tiers[3][4] = {{ca1, la1, ca2, la2}, {cb1, lb1, cb2, lb2}, {cap1, lg1, cap2, lg2}};
    for (int t = 0; t < 3; ++t)
      hipLaunchKernelGGL((k_rap<true>), dim3(grid), dim3(64), ldsz(tiers[t][0], tiers[t][2]), 0, dR, dA.view(),
                         dP.view(), tiers[t][0], tiers[t][1], tiers[t][2], tiers[t][3], len.p, Ci.p, Cj.p, Ca.p,
                         nra.p, t + 1, ca1 / 2, ca2 / 2, cb1 / 2, cb2 / 2);
  } else {
    hipLaunchKernelGGL((k_rap<true>), dim3(grid), dim3(64), lds, 0, dR, dA.view(), dP.view(), cap1, lg1, cap2, lg2,
                       len.p, Ci.p, Cj.p, Ca.p, nullptr, 0, 0, 0, 0, 0);
  }
  SDV(hipGetLastError());
  T.lap("rap fill kernel");
  C.resize_rows(nc, nc);
  C.i = ci;
  Cj.down(C.j, (size_t)ci[nc]);
  Ca.down(C.a, (size_t)ci[nc]);
  for (size_t k = 0; k < ovf.size(); ++k) {
    std::copy(oj[k].begin(), oj[k].end(), C.j.begin() + ci[ovf[k]]);
    std::copy(oa[k].begin(), oa[k].end(), C.a.begin() + ci[ovf[k]]);
  }
  T.lap("C download");
  g_host_rows = (long long)ovf.size();
}

}  // namespace hve
