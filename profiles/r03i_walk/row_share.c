/* Share of steps whose D_t is a learned row, along H1 / H2 sequences of the m = 6 bench
 * models (learn_len 10^6), from the C oracle's own model and streams (measurement tool,
 * not product code): rowfrac, out-of-row segments per 1000 steps and their mean length,
 * the share of wave-steps where all 64 H1 lanes sit in rows, and a log2 histogram of the
 * out-of-row segment lengths.  DESIGN.md "Walk mode" quotes it.
 *   gcc -O2 -fopenmp -I../../oracle -o row_share row_share.c -lm && ./row_share 20000 2 */
#include <stdio.h>
#include "cvd_oracle.c"
int main(int argc, char** argv) {
  const double ps[6] = {0.01, 0.02, 0.05, 0.1, 0.15, 0.2};
  static const uint8_t t1[] = {1,0,1,1,0,1,1, 1,1,1,1,0,0,1};
  static const uint8_t t2[] = {1,1,1,1,0,0,1, 1,0,1,1,0,1,1};
  oc_code c1 = {1, 2, 6, t1}, c2 = {1, 2, 6, t2};
  const int64_t N = argc > 1 ? atoll(argv[1]) : 20000;
  const int W = 64, NS = argc > 2 ? atoi(argv[2]) : 2;   /* waves of 64 H1 seqs */
  Tabs T1, T2; make_tabs(&c1, &T1); make_tabs(&c2, &T2);
  for (int ip = 0; ip < 6; ++ip) {
    double p = ps[ip];
    Model* Mo = oc_model_create(&c1, p, 1000000, 200, 1.0, 12345, 0, 1000000, 0);
    uint32_t tag = oc_grid_tag(N, p);
    for (int h = 0; h < 2; ++h) {
      const Tabs* Te = h ? &T2 : &T1;
      int64_t rowsteps = 0, steps = 0, segs = 0, allrow = 0, wsteps = 0, seglen_hist[8] = {0};
      for (int wv = 0; wv < NS; ++wv) {
        uint8_t D[64][64]; Stream st[64]; int inrow_prev[64]; int64_t runlen[64];
        for (int l = 0; l < W; ++l) { memset(D[l], 0, 64); stream_init(&st[l], Te, 12345, tag, 2 * (uint64_t)(wv * W + l) + h, p); inrow_prev[l] = 1; runlen[l] = 0; }
        for (int64_t t = 0; t < N; ++t) {
          int all = 1;
          for (int l = 0; l < W; ++l) {
            int r = stream_next(&st[l], t);
            uint8_t Dn[64]; oc_step(&Mo->T, D[l], r, Dn); memcpy(D[l], Dn, 64);
            int in = idx_find(&Mo->idx, D[l]) >= 0;
            rowsteps += in; steps++;
            if (!in) { all = 0; if (inrow_prev[l]) { segs++; runlen[l] = 0; } runlen[l]++; }
            else if (!inrow_prev[l]) { int64_t b = runlen[l]; int k = 0; while (b > 1 && k < 7) { b >>= 1; k++; } seglen_hist[k]++; }
            inrow_prev[l] = in;
          }
          allrow += all; wsteps++;
        }
      }
      printf("p=%.2f H%d rows=%ld rowfrac=%.4f segs/seq/1e3steps=%.2f mean_seg=%.2f allrow_wave=%.4f hist(log2)=", p, h + 1,
             (long)Mo->idx.n, (double)rowsteps / steps, 1000.0 * segs / steps, segs ? (double)(steps - rowsteps) / segs : 0.0,
             (double)allrow / wsteps);
      for (int k = 0; k < 8; ++k) printf("%ld ", (long)seglen_hist[k]);
      printf("\n"); fflush(stdout);
    }
    oc_model_destroy(Mo);
  }
  return 0;
}
