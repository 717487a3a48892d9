/* Walk-mode schedule of one H1 wave (cvd_device.h k1b_walk), simulated on the C oracle's
 * own D sequences (measurement tool, not product code).  Per lane the learned-row flags
 * inrow[t] (D_t is a row of the m = 6 bench model, learn_len 10^6) come from the oracle's
 * streams; the simulator then replays k1b_walk's modes (WALK / PEND / ACS / DONE),
 * two-step walk records, bursts of <= 7 iterations and ACS step pairs under the
 * (wmin, amin) rule, and counts ACS iterations (each costs the wave two ACS steps of VALU
 * whatever the number of lanes in them) and burst iterations (one dependent load each).
 * K > 1: each lane takes K sequences in turn (a lane that finishes one starts the next).
 *   gcc -O2 -fopenmp -I../oracle -o walk_sched_sim walk_sched_sim.c -lm
 *   ./walk_sched_sim N p K [wmin amin] */
#include <stdio.h>
#include "cvd_oracle.c"
enum { ACS = 0, PEND = 1, WALK = 2, DONE = 3 };
int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 100000;
  const double p = argc > 2 ? atof(argv[2]) : 0.02;
  const int K = argc > 3 ? atoi(argv[3]) : 1;
  const int wmin = argc > 4 ? atoi(argv[4]) : 48, amin = argc > 5 ? atoi(argv[5]) : 4;
  const int W = 64, burst = 7;
  static const uint8_t t1[] = {1,0,1,1,0,1,1, 1,1,1,1,0,0,1};
  oc_code c1 = {1, 2, 6, t1};
  Tabs T1; make_tabs(&c1, &T1);
  Model* Mo = oc_model_create(&c1, p, 1000000, 200, 1.0, 12345, 0, 1000000, 0);
  const uint32_t tag = oc_grid_tag(N, p);
  const int NS = W * K;
  uint8_t* inrow = malloc((size_t)NS * (N + 1));
#pragma omp parallel for schedule(dynamic)
  for (int s = 0; s < NS; ++s) {
    uint8_t D[64], Dn[64]; memset(D, 0, 64); Stream st; stream_init(&st, &T1, 12345, tag, 2 * (uint64_t)s, p);
    uint8_t* f = inrow + (size_t)s * (N + 1);
    f[0] = 1;
    for (int64_t t = 0; t < N; ++t) {
      oc_step(&Mo->T, D, stream_next(&st, t), Dn); memcpy(D, Dn, 64);
      f[t + 1] = idx_find(&Mo->idx, D) >= 0;
    }
  }
  int mode[64], seq[64]; int64_t pos[64];
  for (int l = 0; l < W; ++l) { mode[l] = WALK; seq[l] = l; pos[l] = 0; }
  int next_seq = W;
  int64_t acs_it = 0, acs_lanes = 0, burst_it = 0, bursts = 0, unpacks = 0, acs_lane_steps = 0;
  const uint8_t* F;
#define INROW(l, t) (inrow[(size_t)seq[l] * (N + 1) + (t)])
  /* a lane at pos == N is done: it takes the next sequence if there is one */
  #define FINISH(l) do { if (pos[l] == N) { if (next_seq < NS) { seq[l] = next_seq++; pos[l] = 0; mode[l] = WALK; } else mode[l] = DONE; } } while (0)
  for (;;) {
    int nA = 0, nW = 0;
    for (int l = 0; l < W; ++l) { nA += mode[l] <= PEND; nW += mode[l] == WALK; }
    if (nA + nW == 0) break;
    if (nW && (nA == 0 || nW >= wmin || nA < amin)) {
      ++bursts;
      for (int b = 0; b < burst; ++b) {
        ++burst_it;
        int any = 0;
        for (int l = 0; l < W; ++l) {
          if (mode[l] != WALK) continue;
          if (pos[l] + 2 <= N) {
            if (!INROW(l, pos[l] + 1)) { mode[l] = PEND; continue; }
            ++pos[l];
            if (pos[l] == N) { FINISH(l); continue; }
            if (!INROW(l, pos[l] + 1)) { mode[l] = PEND; continue; }
            ++pos[l]; FINISH(l);
          } else {
            if (!INROW(l, pos[l] + 1)) { mode[l] = PEND; continue; }
            ++pos[l]; FINISH(l);
          }
        }
        for (int l = 0; l < W; ++l) any |= mode[l] == WALK;
        if (!any) break;
      }
      continue;
    }
    int anyp = 0;
    for (int l = 0; l < W; ++l) if (mode[l] == PEND) { anyp = 1; mode[l] = ACS; }
    unpacks += anyp;
    ++acs_it; acs_lanes += nA;
    for (int k = 0; k < 2; ++k)
      for (int l = 0; l < W; ++l) {
        if (mode[l] != ACS) continue;
        ++pos[l]; ++acs_lane_steps;
        if (pos[l] == N) { FINISH(l); continue; }
        if (INROW(l, pos[l])) mode[l] = WALK;
      }
  }
  int64_t out_steps = 0;
  for (int s = 0; s < NS; ++s) for (int64_t t = 1; t <= N; ++t) out_steps += !inrow[(size_t)s * (N + 1) + t];
  printf("N=%lld p=%.3f K=%d wmin=%d amin=%d seqs=%d: acs_iters=%lld (per 64 seqs %.0f) lanes/acs=%.1f acs_lane_steps=%lld "
         "out_of_row_steps=%lld bursts=%lld burst_iters=%lld (per 64 seqs %.0f) unpacks=%lld\n",
         (long long)N, p, K, wmin, amin, NS, (long long)acs_it, (double)acs_it / K, acs_it ? (double)acs_lanes / acs_it : 0.0,
         (long long)acs_lane_steps, (long long)out_steps, (long long)bursts, (long long)burst_it, (double)burst_it / K,
         (long long)unpacks);
  return 0;
}
