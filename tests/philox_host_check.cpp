// Host check of the product's Philox4x32-10 forms (csrc/cvd_common.h): philox(), the
// B-block philox_blocks under the launch's key pair (PhiloxKeysS) and under the ten round
// keys precomputed for VGPRs (PhiloxKeysV), and the round-by-round philox_round under
// PhiloxKeysV (the fused kernel's pipelined form) -- against the Random123 known-answer
// vectors (kat_vectors, philox4x32_10) and against each other on random counters.  Compiled
// with g++ by tests/test_philox_host.py; the GPU tests check the device forms' streams.
// TEST INFRASTRUCTURE ONLY.
#include <cstdio>

#include "../detecting-convolutional-codes-via-markovian-statistics_amd/csrc/cvd_common.h"

using namespace cvd;

static int fails = 0;
static void check(bool ok, const char* what, int i) {
  if (!ok) {
    std::printf("FAIL %s case %d\n", what, i);
    ++fails;
  }
}

int main() {
  const uint32_t kat[3][10] = {
      {0u, 0u, 0u, 0u, 0u, 0u, 0x6627e8d5u, 0xe169c58du, 0xbc57ac4cu, 0x9b00dbd8u},
      {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x408f276du, 0x41c83b0eu,
       0xa20bc7c6u, 0x6d5451fdu},
      {0x243f6a88u, 0x85a308d3u, 0x13198a2eu, 0x03707344u, 0xa4093822u, 0x299f31d0u, 0xd16cfe09u, 0x94fdccebu,
       0x5001e420u, 0x24126ea1u}};
  for (int i = 0; i < 3; ++i) {
    const uint32_t* v = kat[i];
    const U4 a = philox(v[0], v[1], v[2], v[3], v[4], v[5]);
    check(a.x == v[6] && a.y == v[7] && a.z == v[8] && a.w == v[9], "philox", i);
    uint32_t c1[1][4] = {{v[0], v[1], v[2], v[3]}};
    philox_blocks<1>(c1, PhiloxKeysS{v[4], v[5]});
    check(c1[0][0] == v[6] && c1[0][1] == v[7] && c1[0][2] == v[8] && c1[0][3] == v[9], "blocks/S", i);
    PhiloxKeysV kv;
    kv.init(v[4], v[5]);
    uint32_t c2[1][4] = {{v[0], v[1], v[2], v[3]}};
    philox_blocks<1>(c2, kv);
    check(c2[0][0] == v[6] && c2[0][1] == v[7] && c2[0][2] == v[8] && c2[0][3] == v[9], "blocks/V", i);
    uint32_t c3[1][4] = {{v[0], v[1], v[2], v[3]}};
    for (int r = 0; r < 10; ++r) philox_round<1>(c3, kv, r);
    check(c3[0][0] == v[6] && c3[0][1] == v[7] && c3[0][2] == v[8] && c3[0][3] == v[9], "round/V", i);
  }
  // two blocks at once under each key form = two single calls, on pseudo-random counters
  uint32_t s = 12345u;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s; };
  for (int i = 0; i < 1000; ++i) {
    const uint32_t k0 = rnd(), k1 = rnd();
    uint32_t c[2][4], cs[2][4], cr[2][4];
    for (int b = 0; b < 2; ++b)
      for (int j = 0; j < 4; ++j) c[b][j] = cs[b][j] = cr[b][j] = rnd();
    PhiloxKeysV kv;
    kv.init(k0, k1);
    philox_blocks<2>(c, kv);
    philox_blocks<2>(cs, k0, k1);
    uint32_t a0 = k0, a1 = k1;
    for (int r = 0; r < 10; ++r) {
      philox_round<2>(cr, a0, a1);
      a0 += kPhiloxW0;
      a1 += kPhiloxW1;
    }
    bool ok = true;
    for (int b = 0; b < 2; ++b)
      for (int j = 0; j < 4; ++j) ok = ok && c[b][j] == cs[b][j] && c[b][j] == cr[b][j];
    check(ok, "two blocks V = S = rounds", i);
  }
  if (fails == 0) std::printf("ok philox forms\n");
  return fails == 0 ? 0 : 1;
}
