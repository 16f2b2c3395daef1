/* sched_sim.c -- replay per-lane DBC pc traces (emulator, wb_emu_set_pc_trace) through
 * wave scheduling policies. Tuning aid for the kernel's scheduler, not a test.
 *
 * Lanes are independent instances, so each lane's pc sequence is fixed; a policy only
 * decides which group of lanes (same pc) a wave runs next. A "round" models the kernel:
 * the chosen group runs in lockstep until its lanes split at a branch, a lane ends, it
 * reaches `other` (the lowest waiting pc above the group's start pc), or 1024 taken jumps.
 *
 * build: gcc -O2 -shared -fPIC -o tools/sched_sim.so tools/sched_sim.c
 * policies: 0 min pc; 1 most lanes (ties: min pc); 2 min pc unless the largest group has
 *           >= k x its lanes (k = arg); 3 most lanes among pcs <= the min pc's next
 *           backward-jump region (approximated: most lanes, then merge check).
 *           3 min pc, but a run that takes a backward jump while a waiting group has
 *           >= arg x its lanes ends there and the next round runs the largest group.
 */
#include <stdint.h>
#include <string.h>

typedef struct { uint64_t dispatches, lane_dispatches, rounds; } sim_out;

/* lhead/lend[pc]: the innermost loop around pc (~0: none), for policy 5: the largest
   group (>= arg x the min-pc group) runs when it waits outside the min-pc group's
   innermost loop */
void sched_sim(const uint32_t *trace, const uint64_t *off /*[n+1]*/, uint32_t n, int policy,
               int arg, int arg2, const uint32_t *lhead, const uint32_t *lend, const uint32_t *phead,
               const uint32_t *pend, sim_out *o) {
  memset(o, 0, sizeof *o);
  for (uint32_t w0 = 0; w0 < n; w0 += 64) {
    const uint32_t nl = n - w0 < 64 ? n - w0 : 64;
    uint64_t pos[64], end[64];
    for (uint32_t l = 0; l < nl; l++) { pos[l] = off[w0 + l]; end[l] = off[w0 + l + 1]; }
    int pick_most = 0;
    for (;;) {
      uint32_t pcs[64], cnt[64], ng = 0, minpc = ~0u;
      uint64_t run = 0;
      for (uint32_t l = 0; l < nl; l++) {
        if (pos[l] >= end[l]) continue;
        run |= 1ull << l;
        const uint32_t p = trace[pos[l]];
        if (p < minpc) minpc = p;
        uint32_t g = 0;
        while (g < ng && pcs[g] != p) g++;
        if (g == ng) { pcs[ng] = p; cnt[ng++] = 0; }
        cnt[g]++;
      }
      if (!run) break;
      uint32_t best = 0, mi = 0;
      for (uint32_t g = 0; g < ng; g++) {
        if (pcs[g] == minpc) mi = g;
        if (cnt[g] > cnt[best] || (cnt[g] == cnt[best] && pcs[g] < pcs[best])) best = g;
      }
      uint32_t g = mi;
      if (policy == 1) g = best;
      if (policy == 2 && cnt[best] >= (uint32_t)arg * cnt[mi]) g = best;
      if (policy == 3 && pick_most) g = best;
      if (policy == 6 && lhead[minpc] != ~0u && cnt[best] >= (uint32_t)arg * cnt[mi] &&
          (pcs[best] > lend[minpc] || pcs[best] < lhead[minpc]) &&
          pcs[best] >= phead[minpc] && pcs[best] <= pend[minpc]) g = best;
      if (policy == 7 && lhead[minpc] != ~0u && lhead[pcs[best]] != ~0u &&
          cnt[best] >= (uint32_t)arg * cnt[mi] &&
          (pcs[best] > lend[minpc] || pcs[best] < lhead[minpc])) g = best;
      if (policy == 8 && lhead[minpc] != ~0u && lend[minpc] - lhead[minpc] < (uint32_t)(arg2 >> 8) &&
          cnt[best] >= (uint32_t)arg * cnt[mi] && pcs[best] > lend[minpc]) g = best;
      if (policy == 5 && lhead[minpc] != ~0u && cnt[best] >= (uint32_t)arg * cnt[mi] &&
          (pcs[best] > lend[minpc] || pcs[best] < lhead[minpc])) g = best;
      /* 4: like 2 (k = arg) but only when the min-pc group has <= arg2 >> 8 lanes */
      if (policy == 4 && cnt[mi] <= (uint32_t)(arg2 >> 8) && cnt[best] >= (uint32_t)arg * cnt[mi]) g = best;
      pick_most = 0;
      uint32_t pc = pcs[g];
      uint64_t act = 0;
      for (uint32_t l = 0; l < nl; l++)
        if (((run >> l) & 1) && trace[pos[l]] == pc) act |= 1ull << l;
      uint32_t other = ~0u;
      for (uint32_t l = 0; l < nl; l++)
        if (((run & ~act) >> l) & 1) {
          const uint32_t p = trace[pos[l]];
          if (p > pc && p < other) other = p;
        }
      o->rounds++;
      uint32_t taken = 0;
      for (;;) {
        o->dispatches++;
        o->lane_dispatches += (uint64_t)__builtin_popcountll(act);
        uint32_t np = ~0u;
        int split = 0;
        for (uint32_t l = 0; l < nl; l++) {
          if (!((act >> l) & 1)) continue;
          pos[l]++;
          if (pos[l] >= end[l]) { split = 1; continue; }
          const uint32_t p = trace[pos[l]];
          if (np == ~0u) np = p; else if (p != np) split = 1;
        }
        if (split || np == ~0u) break;
        if (np != pc + 1 && ++taken >= 1024) break;
        if (policy == 3 && np <= pc && (run & ~act)) {
          uint32_t wc[64], wp[64], nw = 0, mx = 0;
          for (uint32_t l = 0; l < nl; l++)
            if ((((run & ~act) >> l) & 1) && pos[l] < end[l]) {
              const uint32_t p = trace[pos[l]];
              uint32_t k = 0;
              while (k < nw && wp[k] != p) k++;
              if (k == nw) { wp[nw] = p; wc[nw++] = 0; }
              if (++wc[k] > mx) mx = wc[k];
            }
          if (mx >= (uint32_t)arg * (uint32_t)__builtin_popcountll(act)) { pick_most = 1; break; }
        }
        if ((arg2 & 255) == 2 && np < pc) {   /* kernel form: only a jump to <= the lowest waiting pc */
          uint32_t low = ~0u;
          for (uint32_t l = 0; l < nl; l++)
            if ((((run & ~act) >> l) & 1) && trace[pos[l]] < low) low = trace[pos[l]];
          if (np <= low) other = low;
        }
        if (arg2 == 1 && np < pc) {   /* recompute the merge point after a backward jump */
          other = ~0u;
          for (uint32_t l = 0; l < nl; l++)
            if (((run & ~act) >> l) & 1) {
              const uint32_t p = trace[pos[l]];
              if (p >= np && p < other) other = p;
            }
        }
        if (np >= other) break;
        pc = np;
      }
    }
  }
}
