// TEST HARNESS ONLY -- the host C++ of the product built with AddressSanitizer and
// UndefinedBehaviorSanitizer (tests/test_sanitizers.py): the input preparation of zg_prep.h
// (Jubjub point decode, small-order checks, multipacking, hSig BLAKE2b, Sprout packing) and the
// 29-bit-digit field products every kernel uses (zg_fq29_gen.h), on the CPU. Never linked into,
// or loaded by, the product library. (The full harness, tests/native/zg_hosttest.hip, is too
// large to build instrumented in the CPU tier's time.)
#include <string.h>
#include "../../zebra_amd/csrc/zg_prep.h"

using namespace zg;

extern "C" {

int zgt_prep_spend(const uint8_t* cv, const uint8_t* anchor, const uint8_t* nf, const uint8_t* rk, uint8_t* in) {
  return prep_spend(cv, anchor, nf, rk, in);
}
int zgt_prep_output(const uint8_t* cv, const uint8_t* cmu, const uint8_t* epk, uint8_t* in) {
  return prep_output(cv, cmu, epk, in);
}
int zgt_hsig(const uint8_t* seed, const uint8_t* nf0, const uint8_t* nf1, const uint8_t* pk, uint8_t* out) {
  prep_hsig(seed, nf0, nf1, pk, out);
  return 0;
}
int zgt_prep_joinsplit(const uint8_t* anchor, const uint8_t* seed, const uint8_t* nfs, const uint8_t* macs,
                       const uint8_t* cms, uint64_t vpub_old, uint64_t vpub_new, const uint8_t* pk, uint8_t* in) {
  prep_joinsplit(anchor, seed, nfs, nfs + 32, macs, macs + 32, cms, cms + 32, vpub_old, vpub_new, pk, in);
  return 0;
}
void zgt_field_mul(int field, const uint32_t* a, const uint32_t* b, uint32_t* r) {
  switch (field) {
    case 0: fq29_mul(r, a, b); break;
    case 1: fq29_sqr(r, a); break;
    case 2: f2_mul29(r, r + 12, a, a + 12, b, b + 12); break;
    case 3: fr29_mul(r, a, b); break;
    default: bq29_mul(r, a, b); break;
  }
}

}  // extern "C"
