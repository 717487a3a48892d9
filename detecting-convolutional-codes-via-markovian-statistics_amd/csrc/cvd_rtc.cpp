// Code-specialised butterfly detector kernels, compiled at run time.
//
// The k = 1, n = 2 butterfly kernel (cvd_device.h) reads each butterfly's
// branch-metric pair from a per-code table with one v_perm_b32.  With the
// decoder code known at compile time the pair is one of four per-step
// registers chosen statically, which removes 2^(m-1) v_perm and the table's
// scalar loads per step.  The decoder is a run-time input (any G1), so the
// specialised kernel is compiled here, once per (device, m, code) per
// process, from the same device source the library is built from (embedded
// by embed_src.py), and loaded as a module.
//
// Compiler: the ROCm toolchain's clang (device-only compile of one kernel,
// about a second), so the code is produced by the same compiler as the
// library.  hipRTC is the fallback: inside a PyTorch process it resolves to
// the comgr bundled with torch (an older LLVM), whose code for this kernel
// spills and runs ~25% slower than the table-driven kernel -- so it is only
// used when no clang is found.  If both fail, the launcher keeps the compiled
// table-driven kernel (same results, slower) and the model records why
// (cvd_model_jit_status; the Python host warns).
//
// Code objects are cached on disk (CVD_JIT_CACHE, else $XDG_CACHE_HOME/cvd_jit,
// else ~/.cache/cvd_jit; CVD_JIT_CACHE=off disables it), keyed by a hash of the
// full kernel source, the target arch, the compiler path and flags, and the
// tuning defines, so a later process with the same decoder skips the compile.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <spawn.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

#include "cvd_internal.h"

#include "cvd_rtc_src.inc"

extern char** environ;

namespace {

std::mutex g_mu;
std::map<std::tuple<int, int, uint64_t, std::string>, std::pair<hipFunction_t, hipFunction_t>> g_cache;

uint64_t fnv1a(const std::string& s, uint64_t h = 0xcbf29ce484222325ull) {
  for (unsigned char c : s) { h ^= c; h *= 0x100000001b3ull; }
  return h;
}

std::string cache_dir() {
  const char* e = std::getenv("CVD_JIT_CACHE");
  if (e && std::string(e) == "off") return "";
  std::string d;
  if (e && e[0]) d = e;
  else if (const char* x = std::getenv("XDG_CACHE_HOME")) d = std::string(x) + "/cvd_jit";
  else if (const char* h = std::getenv("HOME")) d = std::string(h) + "/.cache/cvd_jit";
  else return "";
  // mkdir -p (the parent of a default path may not exist yet)
  for (size_t i = 1; i <= d.size(); ++i)
    if (i == d.size() || d[i] == '/') (void)::mkdir(d.substr(0, i).c_str(), 0755);
  return d;
}

// The prebuilt cache: code objects compiled at build time (cvd_jit_prebuild, run by
// __graft_entry__.build() for the configured codes) in <directory of libcvd.so>/jit, looked up
// before the user cache with the same key; read only (CVD_JIT_PREBUILT=off skips it).
std::string prebuilt_dir() {
  const char* e = std::getenv("CVD_JIT_PREBUILT");
  if (e && std::string(e) == "off") return "";
  Dl_info info;
  if (::dladdr(reinterpret_cast<void*>(&prebuilt_dir), &info) == 0 || !info.dli_fname) return "";
  std::string p = info.dli_fname;
  const size_t slash = p.rfind('/');
  return slash == std::string::npos ? "" : p.substr(0, slash) + "/jit";
}

bool cache_load(const std::string& path, std::vector<char>& code) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  code.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return !code.empty();
}

void cache_store(const std::string& path, const std::vector<char>& code) {
  const std::string tmp = path + ".tmp." + std::to_string(::getpid());
  {
    std::ofstream f(tmp, std::ios::binary);
    if (!f) return;
    f.write(code.data(), (std::streamsize)code.size());
    if (!f) { ::unlink(tmp.c_str()); return; }
  }
  if (::rename(tmp.c_str(), path.c_str()) != 0) ::unlink(tmp.c_str());   // atomic publish
}

// flags of the clang compile (also part of the cache key)
const char* kClangFlags[] = {"-O3", "-std=c++17", "-ffp-contract=off",
                             // ILP-first machine scheduling: 1-2% faster per launch in the
                             // interleaved A/B (profiles/r01g_ab/), same registers, no spills
                             "-mllvm", "--amdgpu-sched-strategy=max-ilp"};

// two entries per code: one model per launch, and several (k1b_multi, cvd_detect_multi);
// the model's variant defines pick the butterfly kernel or its bit-sliced form (k1s)
std::string entry_source(int m, uint64_t xm) {
  char entry[640];
  std::snprintf(entry, sizeof(entry),
                "\nextern \"C\" __global__ __launch_bounds__(cvd_dev::kK1bBlock, cvd_dev::kK1bWavesPerSimd)\n"
                "void cvd_k1b_spec(cvd_dev::ExpArgs a) { cvd_dev::k1b_spec_entry<%d, 0x%016llxull>(a); }\n"
                "extern \"C\" __global__ __launch_bounds__(cvd_dev::kK1bBlock, cvd_dev::kK1bWavesPerSimd)\n"
                "void cvd_k1b_spec_multi(cvd_dev::MultiArgs a) { cvd_dev::k1b_spec_multi_entry<%d, 0x%016llxull>(a); }\n",
                m, (unsigned long long)xm, m, (unsigned long long)xm);
  return entry;
}

bool file_exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

std::string find_clang();
// the cache file name of a code object: a hash of everything the compile depends on
std::string object_name(const std::string& src, const std::string& arch, const std::string& all_defs) {
  std::string keytxt = src + "\n" + arch + "\n" + find_clang() + "\n" + all_defs;
  for (const char* f : kClangFlags) keytxt += std::string("\n") + f;
  char name[64];
  std::snprintf(name, sizeof(name), "/k1b_%016llx.co", (unsigned long long)fnv1a(keytxt));
  return name;
}

std::string find_clang() {
  if (const char* e = std::getenv("CVD_JIT_CLANG")) return e;
  std::vector<std::string> cands;
  if (const char* r = std::getenv("ROCM_PATH")) cands.push_back(std::string(r) + "/lib/llvm/bin/clang++");
  cands.push_back("/opt/rocm/lib/llvm/bin/clang++");
  cands.push_back("/opt/rocm/llvm/bin/clang++");
  for (const auto& c : cands)
    if (file_exists(c)) return c;
  return "";
}

// device-only compile with the toolchain clang -> code object bytes
bool compile_clang(const std::string& src, const std::string& arch, const std::string& defs, std::vector<char>& code,
                   std::string& err) {
  const std::string clang = find_clang();
  if (clang.empty()) { err = "no clang++ found (set CVD_JIT_CLANG)"; return false; }
  char dir_t[] = "/tmp/cvd_jit_XXXXXX";
  const char* dir = ::mkdtemp(dir_t);
  if (!dir) { err = "mkdtemp failed"; return false; }
  const std::string d(dir), in = d + "/k1b_spec.hip", out = d + "/k1b_spec.co", log = d + "/log.txt";
  {
    std::ofstream f(in);
    f << "#include <hip/hip_runtime.h>\n" << src;
  }
  const std::string arch_opt = "--offload-arch=" + arch;
  std::vector<std::string> args = {clang, "-x", "hip", arch_opt, "--offload-device-only", "--no-gpu-bundle-output"};
  for (const char* f : kClangFlags) args.push_back(f);
  for (const char* f : {"-c", in.c_str(), "-o", out.c_str()}) args.push_back(f);
  {   // the model's variant and tuning experiments (CVD_JIT_DEFINES): -D and -mllvm <opt> only
    std::istringstream ds(defs);
    std::string t, o;
    while (ds >> t) {
      if (t.rfind("-D", 0) == 0) {
        args.insert(args.end() - 4, t);
      } else if (t == "-mllvm" && ds >> o) {
        args.insert(args.end() - 4, t);
        args.insert(args.end() - 4, o);
      }
    }
  }
  std::vector<char*> argv;
  for (auto& s : args) argv.push_back(&s[0]);
  argv.push_back(nullptr);
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_addopen(&fa, 1, log.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  posix_spawn_file_actions_adddup2(&fa, 1, 2);
  pid_t pid = 0;
  int status = -1;
  const int rc = ::posix_spawn(&pid, clang.c_str(), &fa, nullptr, argv.data(), environ);
  posix_spawn_file_actions_destroy(&fa);
  if (rc == 0) ::waitpid(pid, &status, 0);
  bool ok = rc == 0 && WIFEXITED(status) && WEXITSTATUS(status) == 0;
  if (ok) {
    std::ifstream f(out, std::ios::binary);
    code.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    ok = !code.empty();
  }
  if (!ok) {
    std::ifstream f(log);
    std::stringstream ss;
    ss << f.rdbuf();
    err = "clang failed: " + ss.str().substr(0, 2000);
  }
  ::unlink(in.c_str()); ::unlink(out.c_str()); ::unlink(log.c_str()); ::rmdir(dir);
  return ok;
}

bool compile_hiprtc(const std::string& src0, const std::string& arch, const std::string& defs, std::vector<char>& code,
                    std::string& err) {
  hiprtcProgram prog;
  // the -D defines as #define lines (hipRTC takes no -mllvm options here)
  std::string src;
  {
    std::istringstream ds(defs);
    std::string t;
    while (ds >> t)
      if (t.rfind("-D", 0) == 0) {
        const std::string d = t.substr(2);
        const size_t eq = d.find('=');
        src += "#define " + (eq == std::string::npos ? d + " 1" : d.substr(0, eq) + " " + d.substr(eq + 1)) + "\n";
      }
  }
  src += src0;
  if (hiprtcCreateProgram(&prog, src.c_str(), "cvd_k1b_spec.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    err = "hiprtcCreateProgram failed";
    return false;
  }
  const std::string arch_opt = "--offload-arch=" + arch;
  const char* opts[] = {arch_opt.c_str(), "-O3", "-std=c++17", "-ffp-contract=off"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    err = std::string("hipRTC compile failed: ") + hiprtcGetErrorString(rc) + "\n" + log.substr(0, 2000);
    return false;
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code.resize(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  return n > 0;
}

}  // namespace

// hipFunction_t of cvd_k1b_spec<m, code> (and of its multi-model entry
// cvd_k1b_spec_multi, same module) on `device`, compiling them on first use.
int cvd::rtc_k1b_function(int device, int m, uint64_t xm, const char* variant_defs, void** fn_out,
                          void** fn_multi_out) {
  *fn_out = nullptr;
  if (fn_multi_out) *fn_multi_out = nullptr;
  if (const char* e = std::getenv("CVD_NO_JIT"))
    if (e[0] && e[0] != '0') { set_error("JIT: disabled by CVD_NO_JIT"); return -1; }
  std::lock_guard<std::mutex> lock(g_mu);
  // the model's variant (e.g. the LDS-resident filter) before the tuning defines; the
  // variant's own macros (block size, LDS filter, pattern table) are the host's to set --
  // the launch geometry and the filter copy follow them -- so CVD_JIT_DEFINES cannot
  // override them
  std::string env_defs;
  if (const char* e = std::getenv("CVD_JIT_DEFINES")) {
    std::istringstream ds(e);
    std::string t;
    while (ds >> t)
      if (t.rfind("-DCVD_K1B_BLOCK", 0) != 0 && t.rfind("-DCVD_K1B_LDSF", 0) != 0 &&
          t.rfind("-DCVD_FILTER_PAT_BITS", 0) != 0 && t.rfind("-DCVD_K1S_PF", 0) != 0)
        env_defs += " " + t;
  }
  const std::string all_defs = std::string(variant_defs ? variant_defs : "") + env_defs;
  const auto key = std::make_tuple(device, m, xm, all_defs);
  auto it = g_cache.find(key);
  if (it != g_cache.end()) {
    *fn_out = (void*)it->second.first;
    if (fn_multi_out) *fn_multi_out = (void*)it->second.second;
    return 0;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { set_error("JIT: device properties"); return -1; }
  std::string arch = prop.gcnArchName;
  const size_t colon = arch.find(':');
  if (colon != std::string::npos) arch = arch.substr(0, colon);

  const std::string src = std::string(kRtcSource) + entry_source(m, xm);
  std::vector<char> code;
  std::string err1, err2;
  const char* via = std::getenv("CVD_JIT_VIA");   // "hiprtc" forces the fallback (tests)
  const bool force_rtc = via && std::string(via) == "hiprtc";
  // on-disk cache of the clang-built code object (and the read-only prebuilt one)
  std::string cpath, ppath;
  if (!force_rtc) {
    const std::string dir = cache_dir(), pdir = prebuilt_dir(), name = object_name(src, arch, all_defs);
    if (!dir.empty()) cpath = dir + name;
    if (!pdir.empty()) ppath = pdir + name;
  }
  auto load = [&](hipFunction_t& fn, hipFunction_t& fnm) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    hipModule_t mod;
    bool loaded = hipModuleLoadData(&mod, code.data()) == hipSuccess;
    if (loaded && hipModuleGetFunction(&fn, mod, "cvd_k1b_spec") != hipSuccess) {
      (void)hipModuleUnload(mod);   // no single-model entry: the module is of no use
      loaded = false;
    }
    // without the multi-model entry the model still runs the specialised kernel, one launch
    // per model (multi_ok checks rtc_fn_multi)
    if (loaded && hipModuleGetFunction(&fnm, mod, "cvd_k1b_spec_multi") != hipSuccess) fnm = nullptr;
    (void)hipSetDevice(cur);
    return loaded;
  };
  hipFunction_t fn, fnm;
  auto done = [&]() {
    g_cache[key] = std::make_pair(fn, fnm);   // modules live for the process (one per device and code)
    *fn_out = (void*)fn;
    if (fn_multi_out) *fn_multi_out = (void*)fnm;
    return 0;
  };
  // Ranks that start together (one process per GPU, the same decoder) compile a variant once:
  // the first takes an exclusive lock on the cache entry, compiles and publishes it; the others
  // wait for the lock and load the published object (8 concurrent compiles made
  // every rank's setup 22.5 s).  The lock is released when `lk` closes.
  struct Lock {
    int fd = -1;
    ~Lock() {
      if (fd >= 0) ::close(fd);   // (closing drops the flock)
    }
  } lk;
  if (!cpath.empty() && std::getenv("CVD_JIT_NOLOCK") == nullptr) {
    lk.fd = ::open((cpath + ".lock").c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
    if (lk.fd >= 0 && ::flock(lk.fd, LOCK_EX) != 0) {
      ::close(lk.fd);
      lk.fd = -1;
    }
  }
  if (!ppath.empty() && cache_load(ppath, code)) {
    if (load(fn, fnm)) return done();
    code.clear();   // (a prebuilt object this device cannot load: the caches below)
  }
  if (!cpath.empty() && cache_load(cpath, code)) {
    if (load(fn, fnm)) return done();
    ::unlink(cpath.c_str());   // unusable cached object: rebuild it
  }
  bool ok = !force_rtc && compile_clang(src, arch, all_defs, code, err1);
  if (ok && !cpath.empty()) cache_store(cpath, code);
  if (!ok) ok = compile_hiprtc(src, arch, all_defs, code, err2);
  if (!ok) { set_error("JIT: " + err1 + " | " + err2); return -1; }
  if (!load(fn, fnm)) { set_error("JIT: module load failed"); return -1; }
  return done();
}

int cvd::rtc_prebuild(int m, uint64_t xm, const char* variant_defs, const char* arch, const char* dir) {
  if (!arch || !dir) { set_error("prebuild: null argument"); return -1; }
  const std::string src = std::string(kRtcSource) + entry_source(m, xm);
  const std::string defs = variant_defs ? variant_defs : "";
  const std::string path = std::string(dir) + object_name(src, arch, defs);
  std::vector<char> code;
  if (cache_load(path, code)) return 0;
  for (size_t i = 1; i <= std::string(dir).size(); ++i)
    if (i == std::string(dir).size() || dir[i] == '/') (void)::mkdir(std::string(dir).substr(0, i).c_str(), 0755);
  std::string err;
  if (!compile_clang(src, arch, defs, code, err)) { set_error("prebuild: " + err); return -1; }
  cache_store(path, code);
  if (!file_exists(path)) { set_error("prebuild: cannot write " + path); return -1; }
  return 0;
}
