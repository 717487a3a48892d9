// Driver of the host sanitizer build: exercises every host-side ABI entry of
// cvd_host.cpp on the BASELINE codes (dense m = 2 and rate-2/3 m = 4, sparse
// m = 6), including the model save/load round trip.  Exit status 0 = clean.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../../include/cvd.h"

namespace {
int fails = 0;
void expect(bool ok, const char* what) {
  if (!ok) { std::fprintf(stderr, "FAIL: %s (%s)\n", what, cvd_last_error()); ++fails; }
}

struct CodeT {
  int k, n, m;
  std::vector<uint8_t> taps;
  cvd_code c() const { return cvd_code{k, n, m, taps.data()}; }
};

void run(const CodeT& ct, double p, int64_t learn_len, const char* path) {
  const cvd_code c = ct.c();
  const int M = 1 << ct.m, K = 1 << ct.k, R = 1 << ct.n;
  std::vector<int32_t> out((size_t)M * K), nxt((size_t)M * K);
  expect(cvd_code_tables(&c, out.data(), nxt.data()) == 0, "code tables");
  std::vector<uint8_t> D((size_t)M, 0), Dn((size_t)M);
  for (int r = 0; r < R; ++r) expect(cvd_metric_step(&c, D.data(), r, Dn.data()) == 0, "metric step");
  int64_t S = 0;
  const int rc = cvd_enumerate(&c, 4000, &S, nullptr, nullptr);
  if (rc == 0) {
    std::vector<uint8_t> st((size_t)S * M);
    std::vector<int32_t> nx((size_t)S * R);
    expect(cvd_enumerate(&c, 4000, &S, st.data(), nx.data()) == 0, "enumerate");
  }
  cvd_learn_params prm{p, learn_len, 200, 1.0, 12345, 4000, 20000};
  cvd_model* mo = nullptr;
  expect(cvd_model_create(&c, &prm, &mo) == 0 && mo, "model create");
  if (!mo) return;
  cvd_model_info inf;
  expect(cvd_model_info_get(mo, &inf) == 0, "info");
  std::vector<double> lp((size_t)inf.n_rows * R);
  std::vector<uint8_t> keys((size_t)inf.n_rows * M);
  expect(cvd_model_rows(mo, lp.data(), keys.data(), inf.n_rows) == 0, "rows");
  if (inf.kind == 0) {
    std::vector<double> P((size_t)inf.S * inf.S);
    expect(cvd_model_dense_P1(mo, P.data(), inf.S) == 0, "dense P1");
  }
  expect(cvd_model_save(mo, path) == 0, "save");
  cvd_model* back = nullptr;
  expect(cvd_model_load(path, &back) == 0 && back, "load");
  if (back) {
    cvd_model_info ib;
    expect(cvd_model_info_get(back, &ib) == 0, "info (loaded)");
    std::vector<double> lp2(lp.size());
    std::vector<uint8_t> k2(keys.size());
    expect(cvd_model_rows(back, lp2.data(), k2.data(), ib.n_rows) == 0, "rows (loaded)");
    expect(ib.n_rows == inf.n_rows && ib.hash_capacity == inf.hash_capacity && ib.max_probe == inf.max_probe &&
               std::memcmp(lp.data(), lp2.data(), lp.size() * sizeof(double)) == 0 && keys == k2,
           "round trip");
    cvd_model_destroy(back);
  }
  expect(cvd_model_upload(mo, 0) != 0, "upload refused without a device");
  cvd_model_destroy(mo);
  std::printf("ok: k=%d n=%d m=%d p=%g kind=%d S=%lld rows=%lld\n", ct.k, ct.n, ct.m, p, inf.kind,
              (long long)inf.S, (long long)inf.n_rows);
}
}  // namespace

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/cvd_asan_model.bin";
  CodeT m2{1, 2, 2, {1, 1, 1, 1, 0, 1}};
  CodeT m6{1, 2, 6, {1, 0, 1, 1, 0, 1, 1, 1, 1, 1, 1, 0, 0, 1}};
  CodeT r23{2, 3, 4, {1, 0, 0, 0, 1, 0, 1, 1, 1, 1, 1, 1, 1, 0, 1, 0, 1, 0, 1, 0, 0, 1, 1, 0, 0, 1, 1, 0, 1, 0}};
  run(m2, 0.05, -1, path);
  run(r23, 0.1, -1, path);
  run(m6, 0.05, 30000, path);
  run(m6, 0.2, -1, path);   // default sparse length (20000 via default_learn_len)
  // bad arguments come back as status codes, not crashes
  cvd_model* mo = nullptr;
  cvd_code bad{1, 2, 9, m2.taps.data()};
  cvd_learn_params prm{0.1, -1, 200, 1.0, 1, 4000, 1000};
  expect(cvd_model_create(&bad, &prm, &mo) != 0 && !mo, "bad shape rejected");
  expect(cvd_model_load("/nonexistent/cvd.bin", &mo) != 0, "missing file rejected");
  std::printf(fails ? "FAILED\n" : "all clean\n");
  return fails ? 1 : 0;
}
