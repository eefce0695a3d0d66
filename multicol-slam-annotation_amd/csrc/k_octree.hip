// K3: DistributeOctTree (src/mdBRIEFextractorOct.cpp:569-861) as an order-exact,
// data-parallel emulation: one 256-thread workgroup per (frame, level); node lists in LDS
// (ping-pong), candidates + their current node in global memory (L2-resident).
#include "common.hpp"
#include "extractor_kernels.hpp"
#include <algorithm>

namespace mcs {

// ===========================================================================
// K3: DistributeOctTree as a data-parallel, order-exact emulation, one workgroup per
// (frame, level).  See DESIGN.md "octree".  The std::list order of the reference is
// reproduced exactly: children are pushed to the front in (node order, n1..n4) order,
// untouched nodes keep their relative order; final-phase node choice follows
// sort(size, pointer) with pointer order pinned to creation order.
// ===========================================================================

constexpr int kOctThreads = 256;

__device__ __forceinline__ int oct_quad(uint32_t pk, int midx, int midy) {
  const int x = pk & 0xFFF, y = (pk >> 12) & 0xFFF;
  return (x >= midx ? 1 : 0) + (y >= midy ? 2 : 0);
}

// CAP: candidates of a (frame, level) kept in LDS when they fit (every subdivision round reads
// them again; from global memory each round was a dependent round trip); larger lists stay in
// global memory.  Both cases go through one generic pointer.
template <int MAXL, int CAP>
__global__ __launch_bounds__(kOctThreads) void k_octree(OctArgs a) {
  constexpr int kOctPer = MAXL / kOctThreads;  // nodes per thread in node scans
  // level-major dispatch: every frame's level-0 list (the longest: most candidates, most
  // nodes, most rounds) is issued before any level-1 list, and so on, so the short upper-level
  // lists fill the tail instead of a few level-0 lists running alone at the end
  const int xb = blockIdx.x & 7, kb = blockIdx.x >> 3, fg = (a.nframes + 7) >> 3;
  const int l = kb / fg, f = xb + 8 * (kb - l * fg);
  if (f >= a.nframes) return;
  const int tid = threadIdx.x;
  const LevelPlan& L = a.lv[l];
  // LDS is what limits residency (workgroups per CU) of this latency-bound kernel, so the
  // tables are sized to their value ranges: positions < MAXL fit int16, flags are 0/1/2;
  // counts stay int (a node may hold tens of thousands of candidates on noise images).
  __shared__ __attribute__((aligned(8))) int s_pref[2 * MAXL];  // cell prefix (<= 2*MAXL cells, launch_octree); then u64 sort keys
  __shared__ int s_scan[2 * (kOctThreads / 64)];   // double-buffered wave totals (block_excl_scan1)
  int scan_par = 0;
  __shared__ int16_t nx0[2][MAXL], ny0[2][MAXL], nx1[2][MAXL], ny1[2][MAXL];
  __shared__ int ncnt[2][MAXL], nseq[2][MAXL];
  __shared__ int ccnt[MAXL * 4];      // child counts; reused for best keys
  __shared__ int16_t npos[MAXL * 4];  // new position per (node, child); kept uses slot 0
  __shared__ uint8_t nflag[MAXL];     // expanding / in-E / processed flags
  __shared__ uint8_t nflag2[MAXL];    // the main loop's next-round flags
  __shared__ int s_var[8];
  __shared__ uint32_t s_cand[CAP > 0 ? CAP : 1];
  __shared__ int32_t s_cnode[CAP > 0 ? CAP : 1];

  uint32_t* const gcand = a.cand + (int64_t)f * a.cand_fstride + L.cand_off;
  int32_t* const gcnode = a.cnode + (int64_t)f * a.cand_fstride + L.cand_off;
  const uint32_t* slots = a.slots + (int64_t)f * a.slots_fstride;
  const int32_t* counts = a.cell_counts + (int64_t)f * a.ncells + L.cell_begin;
  const int nc = L.cell_end - L.cell_begin;
  const int N = L.nfeat;

  // ---- 1. gather candidates of this level in reference (cell, row, col) order
  int n = 0;
  // the cells' slot offsets go to LDS beside the prefix (ccnt is free until the main loop), so
  // a candidate's gather below is one global load instead of two dependent ones
  for (int base = 0; base < nc; base += kOctThreads) {
    const int i = base + tid;
    const int v = i < nc ? counts[i] : 0;
    if (i < nc) ccnt[i] = a.cells[L.cell_begin + i].slot_off;
    int tot;
    const int ex = dev::block_excl_scan1<kOctThreads>(v, s_scan, scan_par, &tot);
    if (i < nc) s_pref[i] = n + ex;
    n += tot;
  }
  __syncthreads();
  const bool inl = n <= CAP;
  uint32_t* const cand = inl ? s_cand : gcand;
  int32_t* const cnode = inl ? s_cnode : gcnode;
  // candidate i of the level: its cell is the last one whose prefix is <= i (empty cells share
  // their successor's prefix), found by binary search in LDS; every candidate's two dependent
  // loads are independent of the others (the per-cell walk chained them cell after cell).
  // The global copy is kept for mcs_extractor_read_stage.
  _Pragma("unroll 2") for (int i = tid; i < n; i += kOctThreads) {
    int lo = 0, hi = nc;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (s_pref[mid] <= i) lo = mid + 1;
      else hi = mid;
    }
    const int c = lo - 1;
    const uint32_t v = slots[ccnt[c] + (i - s_pref[c])];
    cand[i] = v;
    if (inl) gcand[i] = v;
  }
  __syncthreads();

  // ---- 2. initial nodes (:650-683)
  const int nIni = L.nini;
  int cur = 0;
  if (tid < nIni) {
    nx0[0][tid] = (int16_t)(int)(L.hx * (double)tid);
    nx1[0][tid] = (int16_t)(int)(L.hx * (double)(tid + 1));
    ny0[0][tid] = 0;
    ny1[0][tid] = (int16_t)L.height_rel;
    ncnt[0][tid] = 0;
    nseq[0][tid] = tid;
  }
  __syncthreads();
  _Pragma("unroll 4") for (int k = tid; k < n; k += kOctThreads) {
    const int x = cand[k] & 0xFFF;
    const int node = (int)((double)(float)x / L.hx);
    cnode[k] = node;
    atomicAdd(&ncnt[0][node], 1);
  }
  __syncthreads();
  if (tid == 0) {  // erase empty initial nodes, keep order
    int m = 0;
    for (int i = 0; i < nIni; i++) {
      if (ncnt[0][i] > 0) {
        nx0[1][m] = nx0[0][i]; ny0[1][m] = ny0[0][i]; nx1[1][m] = nx1[0][i]; ny1[1][m] = ny1[0][i];
        ncnt[1][m] = ncnt[0][i]; nseq[1][m] = nseq[0][i];
        npos[i] = (int16_t)m++;
      }
    }
    s_var[0] = m;
  }
  __syncthreads();
  cur = 1;
  int Lsz = s_var[0];
  int seqc = nIni;
  // the first round's flags and cleared counts, then the remap to the kept initial nodes and
  // that round's child counting in one pass
  for (int i = tid; i < Lsz; i += kOctThreads) {
    nflag[i] = ncnt[1][i] > 1;
    ccnt[4 * i] = ccnt[4 * i + 1] = ccnt[4 * i + 2] = ccnt[4 * i + 3] = 0;
  }
  __syncthreads();
  _Pragma("unroll 4") for (int k = tid; k < n; k += kOctThreads) {
    const int nn = npos[cnode[k]];
    cnode[k] = nn;
    if (nflag[nn]) {
      const int midx = nx0[1][nn] + ((nx1[1][nn] - nx0[1][nn] + 1) >> 1);
      const int midy = ny0[1][nn] + ((ny1[1][nn] - ny0[1][nn] + 1) >> 1);
      atomicAdd(&ccnt[4 * nn + oct_quad(cand[k], midx, midy)], 1);
    }
  }
  __syncthreads();

  // ---- 3. main subdivision loop (:692-837)
  // When a round is followed by another main-loop round, its candidate update and the next
  // round's child counting are one pass (the next round's flags and cleared counts are set
  // between them): one pass over the candidates and one barrier fewer per round.
  bool finished = false;
  int lastPushBase = 0;
  uint8_t* fl = nflag;     // this round's expanding flags
  uint8_t* fln = nflag2;   // the next round's, set ahead
  bool counted = true;     // this round's child counts came from the previous pass
  while (true) {
    const int prevSize = Lsz;
    const int nxt = cur ^ 1;
    if (!counted) {
      for (int i = tid; i < Lsz; i += kOctThreads) {
        fl[i] = ncnt[cur][i] > 1;
        ccnt[4 * i] = ccnt[4 * i + 1] = ccnt[4 * i + 2] = ccnt[4 * i + 3] = 0;
      }
      __syncthreads();
      _Pragma("unroll 4") for (int k = tid; k < n; k += kOctThreads) {
        const int nd = cnode[k];
        if (fl[nd]) {
          const int midx = nx0[cur][nd] + ((nx1[cur][nd] - nx0[cur][nd] + 1) >> 1);
          const int midy = ny0[cur][nd] + ((ny1[cur][nd] - ny0[cur][nd] + 1) >> 1);
          atomicAdd(&ccnt[4 * nd + oct_quad(cand[k], midx, midy)], 1);
        }
      }
      __syncthreads();
    }
    // per thread: kOctPer consecutive nodes -> pushes (expanding) / kept
    int pushes = 0, kept = 0, expandKids = 0;
    const int i0 = tid * kOctPer;
    for (int j = 0; j < kOctPer; j++) {
      const int i = i0 + j;
      if (i >= Lsz) break;
      if (fl[i]) {
        for (int q = 0; q < 4; q++) {
          const int cq = ccnt[4 * i + q];
          pushes += cq > 0;
          expandKids += cq > 1;
        }
      } else {
        kept++;
      }
    }
    int P, K, E2, pushBase, keptBase;
    if (MAXL <= 512) {
      // one scan of the three counts packed in 10-bit fields: each total is <= MAXL (the list
      // a round builds, P + K, stays <= N <= MAXL, and E2 <= P), so no field carries into the
      // next (3 barriers and one wave scan instead of three of each)
      int T3;
      const int ex = dev::block_excl_scan1<kOctThreads>(pushes | (kept << 10) | (expandKids << 20), s_scan, scan_par, &T3);
      pushBase = ex & 0x3FF; keptBase = (ex >> 10) & 0x3FF;
      P = T3 & 0x3FF; K = (T3 >> 10) & 0x3FF; E2 = (T3 >> 20) & 0x3FF;
    } else {
      pushBase = dev::block_excl_scan1<kOctThreads>(pushes, s_scan, scan_par, &P);
      keptBase = dev::block_excl_scan1<kOctThreads>(kept, s_scan, scan_par, &K);
      dev::block_excl_scan1<kOctThreads>(expandKids, s_scan, scan_par, &E2);
    }
    {
      int s = pushBase, kp = keptBase;
      for (int j = 0; j < kOctPer; j++) {
        const int i = i0 + j;
        if (i >= Lsz) break;
        if (fl[i]) {
          const int x0 = nx0[cur][i], y0 = ny0[cur][i], x1 = nx1[cur][i], y1 = ny1[cur][i];
          const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
          for (int q = 0; q < 4; q++) {
            const int cq = ccnt[4 * i + q];
            if (cq == 0) continue;
            const int pos = P - 1 - s;
            npos[4 * i + q] = (int16_t)pos;
            nx0[nxt][pos] = (int16_t)((q & 1) ? mx : x0);
            nx1[nxt][pos] = (int16_t)((q & 1) ? x1 : mx);
            ny0[nxt][pos] = (int16_t)((q & 2) ? my : y0);
            ny1[nxt][pos] = (int16_t)((q & 2) ? y1 : my);
            ncnt[nxt][pos] = cq;
            nseq[nxt][pos] = seqc + s;
            s++;
          }
        } else {
          const int pos = P + kp;
          npos[4 * i] = (int16_t)pos;
          nx0[nxt][pos] = nx0[cur][i]; nx1[nxt][pos] = nx1[cur][i];
          ny0[nxt][pos] = ny0[cur][i]; ny1[nxt][pos] = ny1[cur][i];
          ncnt[nxt][pos] = ncnt[cur][i];
          nseq[nxt][pos] = nseq[cur][i];
          kp++;
        }
      }
    }
    __syncthreads();
    const int Lnew = P + K;
    // the loop's own exit tests (:826-836), known as soon as the round's totals are
    const bool more = !(Lnew >= N || Lnew == prevSize) && !(Lnew + 3 * E2 > N);
    if (more) {
      for (int i = tid; i < Lnew; i += kOctThreads) {
        fln[i] = ncnt[nxt][i] > 1;
        ccnt[4 * i] = ccnt[4 * i + 1] = ccnt[4 * i + 2] = ccnt[4 * i + 3] = 0;
      }
      __syncthreads();
      _Pragma("unroll 4") for (int k = tid; k < n; k += kOctThreads) {
        const int nd = cnode[k];
        const uint32_t pk = cand[k];
        int nn;
        if (fl[nd]) {
          const int midx = nx0[cur][nd] + ((nx1[cur][nd] - nx0[cur][nd] + 1) >> 1);
          const int midy = ny0[cur][nd] + ((ny1[cur][nd] - ny0[cur][nd] + 1) >> 1);
          nn = npos[4 * nd + oct_quad(pk, midx, midy)];
        } else {
          nn = npos[4 * nd];
        }
        cnode[k] = nn;
        if (fln[nn]) {
          const int midx = nx0[nxt][nn] + ((nx1[nxt][nn] - nx0[nxt][nn] + 1) >> 1);
          const int midy = ny0[nxt][nn] + ((ny1[nxt][nn] - ny0[nxt][nn] + 1) >> 1);
          atomicAdd(&ccnt[4 * nn + oct_quad(pk, midx, midy)], 1);
        }
      }
    } else {
      _Pragma("unroll 4") for (int k = tid; k < n; k += kOctThreads) {
        const int nd = cnode[k];
        if (fl[nd]) {
          const int midx = nx0[cur][nd] + ((nx1[cur][nd] - nx0[cur][nd] + 1) >> 1);
          const int midy = ny0[cur][nd] + ((ny1[cur][nd] - ny0[cur][nd] + 1) >> 1);
          cnode[k] = npos[4 * nd + oct_quad(cand[k], midx, midy)];
        } else {
          cnode[k] = npos[4 * nd];
        }
      }
    }
    lastPushBase = seqc;
    seqc += P;
    Lsz = Lnew;
    cur = nxt;
    __syncthreads();
    if (!more) {
      if (Lsz >= N || Lsz == prevSize) finished = true;
      break;   // finished, or -> final phase
    }
    uint8_t* const t = fl; fl = fln; fln = t;
    counted = true;
  }

  // ---- 4. final phase (:771-836): divide largest nodes first until >= N
  if (!finished) {
    int roundBase = lastPushBase;
    while (true) {
      const int prevSize = Lsz;
      const int nxt = cur ^ 1;
      unsigned long long* keys = reinterpret_cast<unsigned long long*>(s_pref);  // MAXL x u64
      // E = nodes created in the previous round with > 1 key
      int inE = 0;
      const int i0 = tid * kOctPer;
      for (int j = 0; j < kOctPer; j++) {
        const int i = i0 + j;
        if (i < Lsz) inE += (nseq[cur][i] >= roundBase && ncnt[cur][i] > 1);
      }
      int M;
      int eb = dev::block_excl_scan1<kOctThreads>(inE, s_scan, scan_par, &M);
      int M2 = 1;
      while (M2 < M) M2 <<= 1;
      for (int j = 0; j < kOctPer; j++) {
        const int i = i0 + j;
        if (i < Lsz) {
          const bool e = nseq[cur][i] >= roundBase && ncnt[cur][i] > 1;
          nflag[i] = 0;
          ccnt[4 * i] = ccnt[4 * i + 1] = ccnt[4 * i + 2] = ccnt[4 * i + 3] = 0;
          if (e) {
            keys[eb++] = ((unsigned long long)ncnt[cur][i] << 40) |
                         ((unsigned long long)nseq[cur][i] << 12) | (unsigned long long)i;
            nflag[i] = 1;
          }
        }
      }
      __syncthreads();
      // descending order by rank counting (the keys are distinct: they end in the node index):
      // two barriers instead of the bitonic network's log2(M)^2 / 2
      (void)M2;
      {
        unsigned long long mk[kOctPer];
        int rk[kOctPer];
#pragma unroll
        for (int t = 0; t < kOctPer; t++) {
          const int i = tid + t * kOctThreads;
          rk[t] = -1;
          if (i < M) {
            const unsigned long long kv = keys[i];
            int r = 0;
            for (int j = 0; j < M; j++) r += keys[j] > kv;
            mk[t] = kv;
            rk[t] = r;
          }
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < kOctPer; t++)
          if (rk[t] >= 0) keys[rk[t]] = mk[t];
      }
      __syncthreads();
      // child counts of E nodes
      _Pragma("unroll 4") for (int k = tid; k < n; k += kOctThreads) {
        const int nd = cnode[k];
        if (nflag[nd]) {
          const int midx = nx0[cur][nd] + ((nx1[cur][nd] - nx0[cur][nd] + 1) >> 1);
          const int midy = ny0[cur][nd] + ((ny1[cur][nd] - ny0[cur][nd] + 1) >> 1);
          atomicAdd(&ccnt[4 * nd + oct_quad(cand[k], midx, midy)], 1);
        }
      }
      __syncthreads();
      // sorted position j -> delta (nonempty children - 1); processed prefix
      int dsum = 0;
      const int j0 = tid * kOctPer;  // M <= MAXL
      int dl[kOctPer], kl[kOctPer];
      for (int jj = 0; jj < kOctPer; jj++) {
        const int j = j0 + jj;
        dl[jj] = 0; kl[jj] = 0;
        if (j < M) {
          const int nd = (int)(keys[j] & 0xFFF);
          int kids = 0;
          for (int q = 0; q < 4; q++) kids += ccnt[4 * nd + q] > 0;
          kl[jj] = kids;
          dl[jj] = kids - 1;
        }
        dsum += dl[jj];
      }
      int Dtot;
      int dpre = dev::block_excl_scan1<kOctThreads>(dsum, s_scan, scan_par, &Dtot);
      // first j with Lsz + inclusive(delta) >= N -> processed = j+1
      if (tid == 0) s_var[1] = M;
      __syncthreads();
      {
        int run = dpre;
        for (int jj = 0; jj < kOctPer; jj++) {
          const int j = j0 + jj;
          if (j >= M) break;
          run += dl[jj];
          if (Lsz + run >= N) { atomicMin(&s_var[1], j + 1); break; }
        }
      }
      __syncthreads();
      const int Mp = s_var[1];
      int Pn, kbase, kb, Kn;
      if (MAXL <= 512) {
        // mark the processed nodes first, so that the children's and the kept nodes' places
        // come from one packed scan (10-bit fields: both totals stay <= MAXL)
        for (int jj = 0; jj < kOctPer; jj++) {
          const int j = j0 + jj;
          if (j >= Mp) break;
          nflag[(int)(keys[j] & 0xFFF)] = 2;
        }
        __syncthreads();
        int mykids = 0, kept = 0;
        for (int jj = 0; jj < kOctPer; jj++)
          if (j0 + jj < Mp) mykids += kl[jj];
        for (int j = 0; j < kOctPer; j++) {
          const int i = i0 + j;
          if (i < Lsz && nflag[i] != 2) kept++;
        }
        int T2;
        const int ex = dev::block_excl_scan1<kOctThreads>(mykids | (kept << 10), s_scan, scan_par, &T2);
        kbase = ex & 0x3FF; kb = ex >> 10;
        Pn = T2 & 0x3FF; Kn = T2 >> 10;
      } else {
        // pushes of processed sorted nodes (in sorted order, children n1..n4)
        int mykids = 0;
        for (int jj = 0; jj < kOctPer; jj++)
          if (j0 + jj < Mp) mykids += kl[jj];
        kbase = dev::block_excl_scan1<kOctThreads>(mykids, s_scan, scan_par, &Pn);
        for (int jj = 0; jj < kOctPer; jj++) {
          const int j = j0 + jj;
          if (j >= Mp) break;
          nflag[(int)(keys[j] & 0xFFF)] = 2;
        }
        __syncthreads();
        int kept = 0;
        for (int j = 0; j < kOctPer; j++) {
          const int i = i0 + j;
          if (i < Lsz && nflag[i] != 2) kept++;
        }
        kb = dev::block_excl_scan1<kOctThreads>(kept, s_scan, scan_par, &Kn);
      }
      // place the processed nodes' children (sorted order, n1..n4) and the kept nodes after them
      {
        int s = kbase;
        for (int jj = 0; jj < kOctPer; jj++) {
          const int j = j0 + jj;
          if (j >= Mp) break;
          const int nd = (int)(keys[j] & 0xFFF);
          const int x0 = nx0[cur][nd], y0 = ny0[cur][nd], x1 = nx1[cur][nd], y1 = ny1[cur][nd];
          const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
          for (int q = 0; q < 4; q++) {
            const int cq = ccnt[4 * nd + q];
            if (cq == 0) continue;
            const int pos = Pn - 1 - s;
            npos[4 * nd + q] = (int16_t)pos;
            nx0[nxt][pos] = (int16_t)((q & 1) ? mx : x0);
            nx1[nxt][pos] = (int16_t)((q & 1) ? x1 : mx);
            ny0[nxt][pos] = (int16_t)((q & 2) ? my : y0);
            ny1[nxt][pos] = (int16_t)((q & 2) ? y1 : my);
            ncnt[nxt][pos] = cq;
            nseq[nxt][pos] = seqc + s;
            s++;
          }
        }
      }
      for (int j = 0; j < kOctPer; j++) {
        const int i = i0 + j;
        if (i < Lsz && nflag[i] != 2) {
          const int pos = Pn + kb++;
          npos[4 * i] = (int16_t)pos;
          nx0[nxt][pos] = nx0[cur][i]; nx1[nxt][pos] = nx1[cur][i];
          ny0[nxt][pos] = ny0[cur][i]; ny1[nxt][pos] = ny1[cur][i];
          ncnt[nxt][pos] = ncnt[cur][i];
          nseq[nxt][pos] = nseq[cur][i];
        }
      }
      __syncthreads();
      _Pragma("unroll 4") for (int k = tid; k < n; k += kOctThreads) {
        const int nd = cnode[k];
        if (nflag[nd] == 2) {
          const int midx = nx0[cur][nd] + ((nx1[cur][nd] - nx0[cur][nd] + 1) >> 1);
          const int midy = ny0[cur][nd] + ((ny1[cur][nd] - ny0[cur][nd] + 1) >> 1);
          cnode[k] = npos[4 * nd + oct_quad(cand[k], midx, midy)];
        } else {
          cnode[k] = npos[4 * nd];
        }
      }
      roundBase = seqc;
      seqc += Pn;
      Lsz = Pn + Kn;
      cur = nxt;
      __syncthreads();
      if (Lsz >= N || Lsz == prevSize) break;
    }
  }

  // ---- 5. retain the best (first max) key per node, in list order (:839-858)
  unsigned int* best = reinterpret_cast<unsigned int*>(ccnt);
  for (int i = tid; i < Lsz; i += kOctThreads) best[i] = 0u;
  __syncthreads();
  _Pragma("unroll 4") for (int k = tid; k < n; k += kOctThreads) {
    const uint32_t pk = cand[k];
    atomicMax(&best[cnode[k]], ((pk >> 24) << 24) | (0xFFFFFFu - (unsigned)k));
  }
  __syncthreads();
  uint32_t* sel = a.sel + (int64_t)f * a.sel_fstride + L.sel_off;
  for (int i = tid; i < Lsz; i += kOctThreads) sel[i] = cand[0xFFFFFFu - (best[i] & 0xFFFFFFu)];
  if (tid == 0) {
    a.sel_count[(int64_t)f * a.nlevels + l] = Lsz;
    atomicAdd(&a.frame_count[f], Lsz);
  }
}


// candidates kept in LDS per (frame, level): LDS per workgroup sets how many workgroups share
// a CU (160 KB), and this latency-bound kernel lives on residency.  768 (39.5 KB) fits four
// workgroups per CU, where 2048 (49.7 KB) fitted three: octree 0.374 -> 0.348 ms per config-B
// step, although more (frame, level) lists then stay in global memory (1024: 41.5 KB, three
// per CU, 0.394 ms)
#ifndef MCS_OCT_CAP
#define MCS_OCT_CAP 768
#endif
void launch_octree(const OctArgs& a, int max_list, hipStream_t st) {
  const unsigned g = xcd_grid(a.nframes, a.nlevels);
  int max_cells = 0;
  for (int l = 0; l < a.nlevels; l++) max_cells = std::max(max_cells, a.lv[l].cell_end - a.lv[l].cell_begin);
  // s_pref holds 2*MAXL cell prefixes (the plan rejects > kMaxCellsPerLevel = 2048)
  if (max_list <= 512 && max_cells <= 1024)
    hipLaunchKernelGGL((k_octree<512, MCS_OCT_CAP>), dim3(g), dim3(kOctThreads), 0, st, a);
  else
    hipLaunchKernelGGL((k_octree<1024, 0>), dim3(g), dim3(kOctThreads), 0, st, a);
}

}  // namespace mcs
