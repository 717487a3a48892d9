// Internal structures shared by the host setup (cvd_host.cpp) and the HIP
// kernels/launchers (cvd_kernels.hip).  Not part of the ABI.
#pragma once
#include <stdint.h>

#include <array>
#include <string>
#include <vector>

#include "cvd_common.h"
#include "cvd_keys.h"

struct cvd_model {
  cvd::CodeDesc dec;          // decoder trellis (G1; Pd_plotter.py:188 "decoder is fixed to H1")
  int32_t kind = 0;           // 0 dense (BFS index, reference-exact), 1 sparse (learned states)
  int64_t S = 0;              // Laplace denominator state count
  int64_t learn_len_eff = 0;
  double laplace = 1.0;
  double logp1_unseen = 0.0;  // log P̂1 of an unvisited row: log(λ / (S λ))
  double lp_min = 0.0;        // smallest log P̂1 a step can add (early decision bound; set at upload)
  std::vector<double> ltref;  // ltref[c] = log(max(c / 2^n, 1e-300)), c = 0..2^n

  // rows (dense: BFS order; sparse: first-visit order of the learning chain)
  int64_t n_rows = 0;
  std::vector<uint8_t> keys;      // [n_rows][2^m] metric bytes
  std::vector<double> logp1;      // [n_rows][2^n]
  std::vector<uint32_t> rec;      // dense only: [S][2^n] = next_index << 4 | c
  struct NZ { int64_t row, col; double val; };
  std::vector<double> rowsum;     // dense only: numpy row sums of counts + λ
  std::vector<NZ> p1_nz;          // dense only: entries with counts (value = C + λ)
  std::vector<int64_t> visits;    // [n_rows] learning-chain visits counted (t in [burn, L)): the
                                  // device numbers rows by it (hot rows share cache lines)

  // explicit-path hash over nibble-packed keys
  int64_t hcap = 0;               // power of two, 0 = none
  int32_t max_probe = 0;
  std::vector<int64_t> row_next;  // [n_rows][2^n] row index of successor(row, r), -1 if not a row
  std::vector<uint32_t> h_filt;   // [fcap] blocked Bloom filter words (filter_pattern)
  std::vector<uint32_t> h_filt_lds;   // the same filter with 2^kFilterPatBitsLds patterns (LDS kernel), or empty
  int64_t fcap = 0;               // filter words, power of two
  // The directories are kept on the host as their occupied slots only -- the slot index of
  // every row and the row's slot contents, by row -- and expanded on the device at upload
  // (every other slot empty; cvd_kernels.hip upload_model): a 1e6-row model's 2 GiB + 2 GiB of
  // mostly empty slots are never built, zeroed or copied on the host.
  std::vector<uint32_t> h_key_rows;   // [n_rows][h_ssw]: slot contents, nibble-packed metric vector (and,
                                      // interleaved, its record at dword NW); empty slots: kEmptyKey words
  std::vector<uint32_t> h_key_slot;   // [n_rows]: the row's directory slot (< hcap)
  int32_t h_rsw = 0;              // row record stride in dwords (row_words)
  int32_t h_ssw = 0;              // directory slot stride in dwords: nw, or (CVD_SLOT_IL) key + record in one slot
  std::vector<uint32_t> h_row_rows;   // (CVD_SLOT_IL=0) [n_rows][h_rsw] records at the key slot's index of
                                      // a separate [hcap][h_rsw] array: per r, 16 B {log P̂1[r] (f64),
                                      // successor row[r] (i32, -1: none), 0}; empty slots zero
  std::vector<uint32_t> h_drow;   // [n_rows][h_rsw]: the same records dense by row id (table mode),
                                  // dword 3 of entry r = the T_ref count c(r)
  std::vector<uint32_t> h_dkey;   // [n_rows][NW]: row keys (device layout) by device row id
  std::vector<uint32_t> h_t2;     // [n_rows][16][8]: two-step walk records (walking models only)
  // the same records in 8 B (k1s walk with the LDS filter, where they fit: rows < 2^16 and at
  // most 4,096 distinct log P̂1): bits 0-11 / 12-23 the two steps' log P̂1 as indices into
  // h_vtab, 24-39 / 43-58 row after one / two steps + 1, 40-42 / 59-61 their T_ref counts
  std::vector<uint32_t> h_t2c;    // [n_rows][16][2]
  std::vector<double> h_vtab;     // the distinct log P̂1 values (exact doubles)
  // bit-sliced tables of the m = 6 kernel k1s (cvd_bitslice.h, cvd_k1s.h), beside the nibble
  // ones (which the other kernels and the trace path read): the Bloom filter over the
  // canonical digest hash, the directory of 256-B slots {six phase images, record}, and six
  // images per row by device row id
  bool bs = false;
  int32_t bs_pat_bits = 12;       // pattern-table bits of the bit-sliced filter (the kernel's LDS table)
  int64_t bhcap = 0;
  int32_t bmax_probe = 0;
  std::vector<uint32_t> h_bfilt, h_bfilt_lds;   // [fcap] each (the LDS copy only with h_filt_lds)
  std::vector<uint32_t> h_bkey_rows;   // [n_rows][64]: slot contents -- images 8 words x 6 phases,
                                       // records 4 x 4 -- of the [bhcap][64] directory (empty: zero, c = 0)
  std::vector<uint32_t> h_bkey_slot;   // [n_rows]: the row's slot (< bhcap)
  int32_t bs_slot_w = 64;         // dwords per directory slot: 64, or 96 (CVD_BS_SLOT3: three lines
                                  // of {two phase images, the record}; kernel -DCVD_K1S_SLOT3=1)
  std::vector<uint32_t> h_bdkey;  // [n_rows][48]
  // LDS pre-filter of k1s (CVD_K1S_PF): one bit per row at bit pl >> (32 - kBsPfLog2Bits) of
  // its digest hash, 2^kBsPfLog2Bits bits (128 KiB) that a 1,024-thread block keeps in LDS;
  // a lane reads its L2 filter word only where this bit is set (empty: not built)
  std::vector<uint32_t> h_bpf;
  int32_t bs_pf_log2 = 20;        // its size: 2^bs_pf_log2 bits (kBsPfLog2Bits unless CVD_BS_PF_LOG2)
  bool rtc_bs = false;            // the specialised kernel built for this model is k1s
  int32_t slot0 = 0;              // row of D_0 = 0 (always 0)
  std::vector<uint32_t> bmp;      // [2^n/2][2^m][2^k] packed (bm(q0), bm(q1)) branch metrics
  // k = 1 orbit kernel: successor(r ^ g0) = successor(r) with states 2j <-> 2j+1 swapped,
  // so only the representatives rep_0 < rep_1 < ... (r < r ^ g0) get an ACS.
  bool k1_ok = false;
  uint32_t repmap = 0, swmap = 0;  // rep index of r (4 bits per r), r > r ^ g0 (1 bit per r)
  std::vector<uint32_t> bmk1;      // [reps/2][2^m][2] packed (bm(rep 2qp), bm(rep 2qp+1))
  // k = 1, n = 2 single-vector kernel (standard butterfly: tap-0 and tap-m columns
  // both 11): per butterfly j, byte y of bfly[j] = popcount(out(j, 0) ^ y)
  bool k1b_ok = false;
  uint32_t bfly_uni = 0;           // every out(j, 0), j < 2^(m-1), in {00, 11}
  uint32_t bfly_even[4] = {0, 0, 0, 0};   // nibble masks of the butterflies j with out(j, 0) in {00, 11}
  uint64_t bfly_x = 0;             // out(j, 0) in bits 2j..2j+1 (the specialisation key)
  void* rtc_fn = nullptr;          // hipFunction_t of the specialised kernel on `device`, if built
  void* rtc_fn_multi = nullptr;    // its multi-model entry (cvd_detect_multi), same module
  int rtc_block = 256;             // its block size (1,024 with the LDS-resident filter)
  bool rtc_ldsf = false;           // it reads the Bloom filter from dynamic LDS (fcap * 4 bytes)
  bool rtc_pf = false;             // it tests the LDS pre-filter h_bpf before the L2 filter (k1s)
  int64_t rtc_persist_grid = 0;    // k1s: blocks of a persistent (work-queue) launch, 0 = none
  std::string jit_error;           // why the specialised kernel is unavailable (empty if built or n/a)
  std::vector<uint32_t> bfly;      // [2^m / 2]

  // device copies
  int device = -1;
  uint32_t* d_rec = nullptr;
  double* d_logp1 = nullptr;
  double* d_ltref = nullptr;
  uint32_t* d_filt = nullptr;
  uint32_t* d_filt_lds = nullptr;
  uint32_t* d_hkey = nullptr;
  uint32_t* d_hrow = nullptr;
  uint32_t* d_drow = nullptr;
  uint32_t* d_dkey = nullptr;
  uint32_t* d_t2 = nullptr;
  uint32_t* d_t2c = nullptr;
  double* d_vtab = nullptr;
  bool rtc_t2c = false;           // the k1s walk reads d_t2c with the value table in LDS
  uint32_t* d_bfilt = nullptr;
  uint32_t* d_bfilt_lds = nullptr;
  uint32_t* d_bkey = nullptr;
  uint32_t* d_bdkey = nullptr;
  uint32_t* d_bpf = nullptr;
  uint32_t* d_bmp = nullptr;
  uint32_t* d_bmk1 = nullptr;
  uint32_t* d_bfly = nullptr;
  int32_t* d_err = nullptr;       // kernel error flags (k1b_walk's scheduler guard), cvd_model_device_error
};

namespace cvd {

void set_error(const std::string& msg);
std::string last_error_copy();
inline int nib_words(int m) { return (1 << m) >= 8 ? (1 << m) / 8 : 1; }
CVD_HD int row_words(int n) { return row_words_c(1 << n); }

// Nibble packing of a metric vector: state s in nibble s (word s / 8, bits 4*(s % 8)).
void pack_nibbles(const uint8_t* D, int M, uint32_t* out);

// kernel launchers (cvd_kernels.hip)
int launch_generate(const CodeDesc& enc, uint32_t k0, uint32_t k1, uint32_t tag, uint64_t thr,
                    int64_t N, int random_input, int64_t seq_base, int64_t seq_stride,
                    uint32_t* d_r, int64_t pitch, int64_t q0, int64_t count, void* stream);
int launch_detect_table(const cvd_model& M, const uint32_t* d_r, int64_t N, int64_t nseq,
                        int64_t n_h1, double* d_sums, int64_t* d_counts, void* stream, bool early = false);
// the whole trial loop in one kernel (generator + LDS table automaton, no streams in
// HBM): trials [trial_begin, trial_begin + T) of one grid point; CVD_E_UNSUPPORTED if
// the model / codes do not fit it
// the fused kernel applies to the model and measured faster than the two-kernel
// pipeline (small LDS tables: 256-thread blocks); cvd_mc_run's AUTO path uses it then
bool mc_fused_preferred(const cvd_model& M);
// the specialised butterfly kernel runs the model's H1 waves in walk mode (k1b_walk)
bool walk_preferred(const cvd_model& M, bool early = false);
// LDS-resident Bloom filter of the specialised kernel (ldsf_wanted: walking models, and
// bit-sliced lockstep models unless CVD_LDSF_LOCKSTEP=0) of at most ldsf_max_rows rows, whose filter is built with 2^kLdsFilterLog2 words (64 KiB, <= 4
// keys per two-word block, ~0.06% false positives) for 512-thread blocks, two per CU
constexpr int kLdsFilterLog2 = 14;
constexpr int64_t kLdsFilterMaxRows = 32768;
// the LDS filter's size (2^log2 words) and row cap: kLdsFilterLog2 / kLdsFilterMaxRows unless
// CVD_LDSF_LOG2 (13..15; 15: 128 KiB, 1,024-thread blocks) / CVD_LDSF_MAX_ROWS set them
int ldsf_log2(bool bs);
// the k1s LDS pre-filter (cvd_keys.h kBsPfLog2Bits: 128 KiB of dynamic LDS, 1,024-thread
// blocks) for bit-sliced models without the LDS-resident filter, unless CVD_BS_PF=0
bool bs_pf_preferred(const cvd_model& M, bool ldsf);
int64_t ldsf_max_rows(bool bs);
bool ldsf_preferred(const cvd_model& M);
// the model is a candidate for the whole Bloom filter in LDS: it walks, or (CVD_LDSF_LOCKSTEP,
// default 1 for bit-sliced models, 0 otherwise) any model small enough, whose lockstep lanes then read the LDS filter instead of the
// pre-filter and the L2 filter
bool ldsf_wanted(const cvd_model& M);
int launch_mc_fused(const cvd_model& M, const CodeDesc& e1, const CodeDesc& e2, uint32_t k0, uint32_t k1,
                    uint32_t tag, uint64_t thr, int64_t N, int64_t trial_begin, int64_t T, double* d_sums,
                    int64_t* d_counts, void* stream, bool early);
int launch_detect_explicit(const cvd_model& M, const uint32_t* d_r, int64_t N, int64_t nseq,
                           int64_t n_h1, double* d_sums, int64_t* d_counts, uint8_t* d_trace,
                           void* stream, int variant, bool early = false);
// launch_detect_explicit variants
constexpr int kExplicitBest = 0, kExplicitOrbit = 1, kExplicitGeneric = 2, kExplicitButterfly = 3;
int upload_model(cvd_model& M, int device);
// CVD_KERNEL_* that launch_detect_explicit(kExplicitBest) picks for this model
int explicit_kernel_of(const cvd_model& M);
// hipRTC-compiled code-specialised butterfly kernel (cvd_rtc.cpp); 0 = ok
// CVD_OK if the model is uploaded to the current device
int check_device(const cvd_model& M);
int rtc_k1b_function(int device, int m, uint64_t xm, const char* variant_defs, void** fn_out,
                     void** fn_multi_out = nullptr);
// the -D set of a specialised-kernel variant (upload_model, and cvd_jit_prebuild: the same text
// keys the same code object)
std::string rtc_variant_defs(int block, bool ldsf, int patbits, bool bs, bool pf, int pf_log2, bool slot3 = false);
// compile one variant for `arch` into `dir` (the prebuilt cache rtc_k1b_function reads first);
// 0 = ok (or already there)
int rtc_prebuild(int m, uint64_t xm, const char* variant_defs, const char* arch, const char* dir);
void free_model_device(cvd_model& M);
bool explicit_supported(int m, int k, int n);
// the model gets the bit-sliced tables and kernel (m = 6 standard-butterfly codes;
// CVD_BITSLICE=0 turns it off)
bool bitslice_preferred(const cvd_model& M);
// id of the multi-model launch variant (cvd_model_info.multi_variant; cvd_kernels.hip)
int64_t multi_variant(const cvd_model& M);
// sequences above which a launch of the model is persistent (cvd_model_info.persist_seqs; 0:
// never), and the block count of such a launch over nseq sequences (0: a block launch)
int64_t persist_seqs(const cvd_model& M);
// the last detect call's chunked launches (cvd_kernels.hip): {chunked groups,
// chunks per sequence C, steps per chunk L, sequences rerun sequentially}; cvd_chunk_last
extern std::array<int64_t, 4> ck_last;
int64_t persist_grid(const cvd_model& M, int64_t nseq);

// P̂1 learning chain on the GPU (cvd_learn.hip): identical outputs to the host chain.
struct LearnStats {
  int64_t mismatched_blocks = 0;   // speculative blocks whose start failed verification
  int64_t fix_passes = 0;          // re-run passes
  int64_t sequential_blocks = 0;   // blocks re-run one by one (cascading mismatches)
  int64_t hash_attempts = 0;       // sort passes (>1: a 64-bit key-hash collision was seen)
  double seconds = 0.0;
  double sequential_seconds = 0.0; // time of the sequential tail (0 unless it ran)
  int64_t host_fallback = 0;       // 1: the GPU chain refused (shape, length, device memory), host chain ran
};
// sparse model: rows = distinct D_0..D_L in first-visit order (keys_out [S][2^m]
// bytes), cnt_out[S][2^n] = transitions over t in [burn, L)
int device_learn_sparse(const CodeDesc& dec, int64_t L, int64_t burn, uint64_t seed, double p, int device,
                        void* stream, std::vector<uint8_t>& keys_out, std::vector<int64_t>& cnt_out,
                        int64_t& S_out, LearnStats* stats);
// dense model: the chain on the BFS automaton next[S][2^n] from index 0
int device_learn_dense(const CodeDesc& dec, const std::vector<int32_t>& next, int64_t S, int64_t L, int64_t burn,
                       uint64_t seed, double p, int device, void* stream, std::vector<int64_t>& cnt_out,
                       LearnStats* stats);

}  // namespace cvd
