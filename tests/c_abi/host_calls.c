/* The drop-in boundary from plain C (include/cvd.h): a C99 program that
 * includes the header, links libcvd.so and makes the host-only calls a maintainer's binding
 * would make first -- version, code tables (viterbi_markov.py:82-106), the model's host build
 * (Pd_plotter.py:123-169) and its info, the chunk diagnostic, error reporting.  No GPU.
 * Test infrastructure: tests/test_c_abi_host.py compiles and runs it. */
#include <stdio.h>
#include <string.h>

#include "cvd.h"

int main(void) {
  if (cvd_version() != CVD_ABI_VERSION) { printf("abi %d != %d\n", cvd_version(), CVD_ABI_VERSION); return 1; }
  /* (7,5) as [n][k][m+1] delay-ordered taps: outputs 1+D+D^2 and 1+D^2 */
  uint8_t taps[] = {1, 1, 1, 1, 0, 1};
  cvd_code g = {1, 2, 2, taps};
  int32_t out[8];
  int32_t nxt[8];
  if (cvd_code_tables(&g, out, nxt) != CVD_OK) { printf("tables: %s\n", cvd_last_error()); return 1; }
  /* out[s*2^k + U]: state 0 -> words 0 (U = 0) and 3 (U = 1), state 1 -> words 1 and 2 */
  printf("out %d %d %d %d next %d %d\n", out[0], out[1], out[2], out[3], nxt[0], nxt[1]);
  cvd_learn_params lp;
  memset(&lp, 0, sizeof lp);
  lp.p = 0.05; lp.learn_len = -1; lp.learn_burn = 200; lp.laplace = 1.0; lp.seed = 12345;
  lp.enum_cap = 500000; lp.default_learn_len = 1000000;
  cvd_model* M = NULL;
  if (cvd_model_create(&g, &lp, &M) != CVD_OK) { printf("create: %s\n", cvd_last_error()); return 1; }
  cvd_model_info info;
  if (cvd_model_info_get(M, &info) != CVD_OK) { printf("info: %s\n", cvd_last_error()); return 1; }
  printf("kind %d S %lld rows %lld\n", (int)info.kind, (long long)info.S, (long long)info.n_rows);
  int64_t ck[4] = {-1, -1, -1, -1};
  if (cvd_chunk_last(ck) != CVD_OK) return 1;
  printf("chunk %lld\n", (long long)ck[0]);
  /* errors come back as status codes with a message, never as exceptions */
  cvd_code bad = {1, 2, 2, NULL};
  const int rc = cvd_code_tables(&bad, out, nxt);
  printf("bad %d %s\n", rc, rc == CVD_E_INVALID && strlen(cvd_last_error()) > 0 ? "ok" : "?");
  cvd_model_destroy(M);
  return 0;
}
