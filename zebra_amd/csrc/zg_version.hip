// zg_version(): the library's identity, including the hash of the exact sources it was compiled
// from (FNV-1a 64 over csrc/*.hip, csrc/*.h and include/zg.h, computed by zebra_amd/build.py or
// rust/verification/build.rs and passed as ZG_SOURCE_HASH), so a test run on the GPU box can
// prove that the library it loaded is the one built from the tree it runs in.
#ifndef ZG_SOURCE_HASH
#error "zg_version.hip is compiled with -DZG_SOURCE_HASH=\"<16 hex digits>\" (zebra_amd/build.py)"
#endif

extern "C" const char* zg_version(void) { return "zebra_amd zg 0.3 gfx950 src " ZG_SOURCE_HASH; }
