// Host-only ASan/UBSan build of cvd_host.cpp (`make asan`): the device-side
// entry points it calls are replaced by these stand-ins, so the BFS, the
// learning chain, the P̂1 rows, the row tables and the model file I/O run under
// the sanitizers without a GPU.  Test harness, not product code.
#include "../cvd_internal.h"
#include "../../../include/cvd.h"

int cvd::upload_model(cvd_model&, int) {
  cvd::set_error("no device in the host sanitizer build");
  return CVD_E_UNSUPPORTED;
}
void cvd::free_model_device(cvd_model&) {}
int cvd::explicit_kernel_of(const cvd_model& M) { return M.k1b_ok ? CVD_KERNEL_BUTTERFLY : CVD_KERNEL_NONE; }
bool cvd::mc_fused_preferred(const cvd_model&) { return false; }
bool cvd::walk_preferred(const cvd_model&, bool) { return false; }
bool cvd::ldsf_preferred(const cvd_model&) { return false; }
bool cvd::ldsf_wanted(const cvd_model&) { return false; }
int64_t cvd::multi_variant(const cvd_model&) { return 0; }
int64_t cvd::persist_seqs(const cvd_model&) { return 0; }
int64_t cvd::persist_grid(const cvd_model&, int64_t) { return 0; }
int cvd::device_learn_sparse(const CodeDesc&, int64_t, int64_t, uint64_t, double, int, void*, std::vector<uint8_t>&,
                             std::vector<int64_t>&, int64_t&, LearnStats*) {
  cvd::set_error("no device in the host sanitizer build");
  return CVD_E_UNSUPPORTED;
}
int cvd::device_learn_dense(const CodeDesc&, const std::vector<int32_t>&, int64_t, int64_t, int64_t, uint64_t, double,
                            int, void*, std::vector<int64_t>&, LearnStats*) {
  cvd::set_error("no device in the host sanitizer build");
  return CVD_E_UNSUPPORTED;
}
std::string cvd::rtc_variant_defs(int, bool, int, bool, bool, int, bool) { return ""; }
int cvd::rtc_prebuild(int, uint64_t, const char*, const char*, const char*) {
  cvd::set_error("no JIT in the host sanitizer build");
  return -1;
}
