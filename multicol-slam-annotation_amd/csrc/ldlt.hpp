// Dense LDL^T factor + solve of the reduced camera system on gfx950 (FP64 matrix cores).
//
// Replaces LinearSolverEigen::solve (ThirdParty/g2o/g2o/solvers/linear_solver_eigen.h:94-126,
// Eigen SimplicialLDLT without pivoting; an exact zero pivot fails the solve) for the Schur
// complement produced by BlockSolver<6,3>::solve (block_solver.hpp:354-486).
//
// Storage: the symmetric matrix is held as its lower 64x64 tiles in diagonal-major order --
// diagonal d = I - J (d = 0: the T diagonal tiles, then the T - 1 tiles of the first
// sub-diagonal, ...), J ascending along a diagonal -- each tile row-major.  A banded system
// (the reduced camera system of keyframes that share points with their neighbours) keeps all
// of its non-zero tiles in one leading range, so the sharded exchange reduces just that range
// (ba.hip).  n is padded to Np = 64 T with an identity block (zero right-hand side), which
// leaves the solution of the leading n x n system unchanged.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <vector>

namespace mcs {
namespace ldlt {

constexpr int TB = 64;

// tiles on the diagonals 0 .. d-1 of a T x T tile triangle
__host__ __device__ inline size_t band_tiles(int d, int T) {
  return (size_t)d * T - (size_t)d * (d - 1) / 2;
}
__host__ __device__ inline size_t toff(int I, int J, int T) {
  return (band_tiles(I - J, T) + J) * (TB * TB);
}
// element (r, c) with r >= c (callers never address the strict upper triangle of a
// diagonal tile through this)
__host__ __device__ inline size_t sidx(int r, int c, int T) {
  return toff(r / TB, c / TB, T) + (size_t)(r % TB) * TB + (c % TB);
}
inline int tiles_for(int n) { return (n + TB - 1) / TB; }
inline size_t tile_doubles(int T) { return (size_t)T * (T + 1) / 2 * TB * TB; }

struct Work {
  double* L;      // tile_doubles(T): off-diagonal L blocks (I > J)
  double* Linv;   // T * 64 * 64: inverse of each unit-lower diagonal L block
  double* z;      // 64 T: D^-1 L^-1 b
  // pipelined factorisation (one launch, see ldlt.hip), set up by pipe_prepare for one T;
  // without it solve() runs one k_panel launch per step
  double* W = nullptr;        // tile_doubles(T): W_ik = L_ik D_k
  double* du = nullptr;       // T * 128: D_k, u_k
  unsigned* sync = nullptr;   // pipe_sync_words(T): ticket, error, product counters, flags
  int4* tasks = nullptr;      // task table
  int ntasks = 0;
  int pipe_T = 0;
  // tile bandwidth of the pipelined factorisation: tiles (I, J) with I - J >= band are zero in A
  // (and stay zero in L: a banded matrix factors without fill outside its band), so no task
  // touches them.  0 = dense (band = T).
  int band = 0;
  bool per_step = false;      // with the pipeline's sync words: one k_panel launch per step
};

// largest tile count of a DENSE pipelined factorisation (task table ~T^3/6 entries); a banded one
// (band D) has ~T D^2 / 2 tasks and is limited by kPipeMaxTasks / kPipeMaxTBand instead
constexpr int kPipeMaxT = 96;
constexpr int kPipeMaxTBand = 4096;
constexpr size_t kPipeMaxTasks = (size_t)1 << 22;
// the band the pipelined path runs with (D clamped to [2, T]; 0 = dense)
inline int pipe_band(int T, int D) { return (D <= 0 || D >= T) ? T : (D < 2 ? 2 : D); }
// whether the pipelined path takes T tiles of band D (task count and tile-count bounds)
bool pipe_supported(int T, int D);
size_t pipe_sync_words(int T, int D = 0);
hipError_t pipe_prepare(Work& w, int T, hipStream_t st, int D = 0);   // allocates W, du, sync, tasks
// the task table for T tiles of band D (host copy, cached for the process: a valid async-copy
// source)
const std::vector<int4>& pipe_tasks_host(int T, int D = 0);
void pipe_release(Work& w);

// Solve status bits in *flag (device; callers clear it, the kernels only OR bits in):
//   kFlagZeroPivot: an exact zero pivot (the reference's failed solve, g2o rejects the trial);
//   kFlagTimeout:   a hand-off wait of the pipelined factorisation / backward substitution gave
//                   up (kernels on other streams holding its workgroups off the CUs, preemption,
//                   profiler serialisation).  x is garbage; the caller must report an error, never
//                   treat it as a rejected trial.
constexpr int kFlagZeroPivot = 1;
constexpr int kFlagTimeout = 2;
// hand-off wait bound in ticks of the 100 MHz real-time counter (default 25,000,000 = 0.25 s);
// a test hook (mcs_ldlt_set_wait_ticks) lowers it to force the timeout path
void set_wait_ticks(long long ticks);
long long wait_ticks();

// A: tiles (destroyed), b: 64 T (destroyed), x: 64 T (out).  Status bits into *flag (above).
// All launches on st.
// skip (nullable, device): every kernel returns at once when *skip != 0 (a device-driven
// optimisation loop that has ended, ba.hip).
hipError_t solve(double* A, double* b, double* x, int T, const Work& w, int* flag, hipStream_t st,
                 const int* skip = nullptr);

// Padding rows/columns [n, 64T): diagonal = diag_value, rest 0; b[n..64T) = 0.
hipError_t pad(double* A, double* b, int n, int T, double diag_value, hipStream_t st,
               const int* skip = nullptr);
// pad + solve of a one-tile system (n <= 64) in one launch, bitwise equal to pad + solve
// (diag_value: the padding diagonal after any exchange, i.e. 1)
// dynamic-LDS limit of a kernel above 64 KB, once per (kernel, device)
hipError_t set_lds_limit(const void* fn, int bytes);

hipError_t solve_one_tile(const double* A, const double* b, double* x, int n, double diag_value, int* flag,
                          hipStream_t st, const int* skip = nullptr);

}  // namespace ldlt
}  // namespace mcs
