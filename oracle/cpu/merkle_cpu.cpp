// ORACLE / CPU BASELINE (test and bench infrastructure only; never linked into the product):
// a C++ restatement of the reference's note-commitment tree path as the
// reference runs it on the CPU, one hash after another:
//   * crypto/src/lib.rs:188-198 sha256_compress; crypto/src/lib.rs:250-275 pedersen_hash with
//     sapling-crypto's algorithm (not vendored; oracle/merkle.py restates it): per segment the
//     3-bit chunk digits summed in Fs, then the exp-table sum of that scalar's bytes (window 8,
//     table[w][i] = i 2^(8 w) G_j, extended-coordinate additions), the affine u via one
//     inversion (binary extended Euclid, as pairing's Fr::inverse)
//   * storage/src/tree_state.rs:193-264 TreeState append / root, one root per mark
// The Pedersen generators come from oracle/merkle.py (mc_init) so this file needs no BLAKE2s.
// Built by oracle/cpu/build.py into oracle/_build/libzgmerkle.so.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

typedef unsigned __int128 u128;

namespace {

// ---- 4 x 64-bit Montgomery arithmetic over a 255-bit modulus
struct Mod {
  uint64_t p[4];
  uint64_t inv;  // -p^-1 mod 2^64
  uint64_t r2[4];
};
// Fr (BLS12-381 scalar field = Jubjub base field)
const Mod FR = {{0xffffffff00000001ULL, 0x53bda402fffe5bfeULL, 0x3339d80809a1d805ULL, 0x73eda753299d7d48ULL},
                0xfffffffeffffffffULL,
                {0xc999e990f3f29c6dULL, 0x2b6cedcb87925c23ULL, 0x05d314967254398fULL, 0x0748d9d99f59ff11ULL}};

struct F {
  uint64_t v[4];
};

bool geq(const uint64_t* a, const uint64_t* b) {
  for (int i = 3; i >= 0; i--)
    if (a[i] != b[i]) return a[i] > b[i];
  return true;
}
void sub_in(uint64_t* a, const uint64_t* b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a[i] - b[i] - br;
    a[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
}
F add(const Mod& m, const F& a, const F& b) {
  F r;
  uint64_t c = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a.v[i] + b.v[i] + c;
    r.v[i] = (uint64_t)t;
    c = (uint64_t)(t >> 64);
  }
  if (c || geq(r.v, m.p)) sub_in(r.v, m.p);
  return r;
}
F sub(const Mod& m, const F& a, const F& b) {
  F r;
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a.v[i] - b.v[i] - br;
    r.v[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
  if (br) {
    uint64_t c = 0;
    for (int i = 0; i < 4; i++) {
      u128 t = (u128)r.v[i] + m.p[i] + c;
      r.v[i] = (uint64_t)t;
      c = (uint64_t)(t >> 64);
    }
  }
  return r;
}
F neg(const Mod& m, const F& a) {
  F z = {{0, 0, 0, 0}};
  return sub(m, z, a);
}
F mul(const Mod& m, const F& a, const F& b) {  // CIOS
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 4; j++) {
      u128 x = (u128)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    u128 x = (u128)t[4] + c;
    t[4] = (uint64_t)x;
    t[5] = (uint64_t)(x >> 64);
    const uint64_t k = t[0] * m.inv;
    x = (u128)k * m.p[0] + t[0];
    c = (uint64_t)(x >> 64);
    for (int j = 1; j < 4; j++) {
      x = (u128)k * m.p[j] + t[j] + c;
      t[j - 1] = (uint64_t)x;
      c = (uint64_t)(x >> 64);
    }
    x = (u128)t[4] + c;
    t[3] = (uint64_t)x;
    t[4] = t[5] + (uint64_t)(x >> 64);
  }
  F r = {{t[0], t[1], t[2], t[3]}};
  if (t[4] || geq(r.v, m.p)) sub_in(r.v, m.p);
  return r;
}
F to_mont(const Mod& m, const F& a) {
  F r2 = {{m.r2[0], m.r2[1], m.r2[2], m.r2[3]}};
  return mul(m, a, r2);
}
F from_mont(const Mod& m, const F& a) {
  F one = {{1, 0, 0, 0}};
  return mul(m, a, one);
}
bool is_zero(const F& a) { return !(a.v[0] | a.v[1] | a.v[2] | a.v[3]); }

// plain-residue inverse by binary extended Euclid (x < p, p odd); montgomery: (aR)^-1 R^2
F inv_plain(const Mod& m, const F& x) {
  uint64_t u[4], v[4];
  memcpy(u, x.v, 32);
  memcpy(v, m.p, 32);
  F b = {{1, 0, 0, 0}}, c = {{0, 0, 0, 0}};
  auto is_one = [](const uint64_t* a) { return a[0] == 1 && !(a[1] | a[2] | a[3]); };
  auto shr1 = [](uint64_t* a) {
    for (int i = 0; i < 3; i++) a[i] = (a[i] >> 1) | (a[i + 1] << 63);
    a[3] >>= 1;
  };
  auto half = [&](F& t) {  // t / 2 mod p
    uint64_t carry = 0;
    if (t.v[0] & 1) {
      uint64_t c2 = 0;
      for (int i = 0; i < 4; i++) {
        u128 s = (u128)t.v[i] + m.p[i] + c2;
        t.v[i] = (uint64_t)s;
        c2 = (uint64_t)(s >> 64);
      }
      carry = c2;
    }
    shr1(t.v);
    t.v[3] |= carry << 63;
  };
  if (is_zero(x)) return x;
  while (!is_one(u) && !is_one(v)) {
    while (!(u[0] & 1)) {
      shr1(u);
      half(b);
    }
    while (!(v[0] & 1)) {
      shr1(v);
      half(c);
    }
    if (geq(u, v)) {
      sub_in(u, v);
      b = sub(m, b, c);
    } else {
      sub_in(v, u);
      c = sub(m, c, b);
    }
  }
  return is_one(u) ? b : c;
}

// ---- Jubjub (a = -1, d = -10240/10241), extended coordinates
struct P4 {
  F x, y, z, t;
};
F D_M;    // d (Montgomery)
F ONE_M;  // 1 (Montgomery)

P4 pt_zero() { return {F{{0, 0, 0, 0}}, ONE_M, ONE_M, F{{0, 0, 0, 0}}}; }
P4 pt_add(const P4& p, const P4& q) {  // sapling-crypto edwards::Point::add (hwcd, a = -1)
  const F a = mul(FR, p.x, q.x);
  const F b = mul(FR, p.y, q.y);
  const F c = mul(FR, mul(FR, D_M, p.t), q.t);
  const F d = mul(FR, p.z, q.z);
  const F h = add(FR, b, a);
  const F e = sub(FR, sub(FR, mul(FR, add(FR, p.x, p.y), add(FR, q.x, q.y)), a), b);
  const F f = sub(FR, d, c);
  const F g = add(FR, d, c);
  return {mul(FR, e, f), mul(FR, g, h), mul(FR, f, g), mul(FR, e, h)};
}

// Fs = Z / r_J, plain residues (digit sums only)
const uint64_t RJ[4] = {0xd0970e5ed6f72cb7ULL, 0xa6682093ccc81082ULL, 0x06673b0101343b00ULL, 0x0e7db4ea6533afa9ULL};
const Mod FS = {{RJ[0], RJ[1], RJ[2], RJ[3]}, 0, {0, 0, 0, 0}};

std::vector<P4> g_table;  // [gen][window][256]
const int WINDOWS = 32;   // ceil(252 / 8)
bool g_ready = false;

P4 from_affine(const uint8_t* xy) {
  F x, y;
  memcpy(x.v, xy, 32);
  memcpy(y.v, xy + 32, 32);
  x = to_mont(FR, x);
  y = to_mont(FR, y);
  return {x, y, ONE_M, mul(FR, x, y)};
}

P4 pedersen_point(const std::vector<uint8_t>& bits) {
  P4 result = pt_zero();
  size_t pos = 0;
  int seg = 0;
  while (pos < bits.size()) {
    F acc = {{0, 0, 0, 0}}, cur = {{1, 0, 0, 0}};
    for (int ch = 0; ch < 63 && pos < bits.size(); ch++) {
      const int a = bits[pos], b = pos + 1 < bits.size() ? bits[pos + 1] : 0, c = pos + 2 < bits.size() ? bits[pos + 2] : 0;
      pos += 3;
      F tmp = cur;
      if (a) tmp = add(FS, tmp, cur);
      cur = add(FS, cur, cur);
      if (b) tmp = add(FS, tmp, cur);
      if (c) tmp = neg(FS, tmp);
      acc = add(FS, acc, tmp);
      cur = add(FS, cur, cur);
      cur = add(FS, cur, cur);
      cur = add(FS, cur, cur);
    }
    // exp-table sum over the scalar's bytes (sapling-crypto pedersen_hash, window 8)
    P4 tmp = pt_zero();
    const P4* tab = &g_table[(size_t)seg * WINDOWS * 256];
    for (int w = 0; w < WINDOWS && !is_zero(acc); w++) {
      const int i = (int)(acc.v[0] & 0xff);
      tmp = pt_add(tmp, tab[w * 256 + i]);
      for (int k = 0; k < 3; k++) acc.v[k] = (acc.v[k] >> 8) | (acc.v[k + 1] << 56);
      acc.v[3] >>= 8;
    }
    result = pt_add(result, tmp);
    seg++;
  }
  return result;
}

void pedersen_merkle(const uint8_t* l, const uint8_t* r, int depth, uint8_t* out) {
  std::vector<uint8_t> bits;
  bits.reserve(516);
  for (int i = 0; i < 6; i++) bits.push_back((depth >> i) & 1);
  for (int i = 0; i < 255; i++) bits.push_back((l[i >> 3] >> (i & 7)) & 1);
  for (int i = 0; i < 255; i++) bits.push_back((r[i >> 3] >> (i & 7)) & 1);
  const P4 p = pedersen_point(bits);
  // into_xy: x = X / Z
  const F zi = inv_plain(FR, from_mont(FR, p.z));
  const F x = mul(FR, from_mont(FR, p.x), to_mont(FR, zi));
  memcpy(out, x.v, 32);
}

// ---- SHA-256 compression (one block, no padding)
const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
inline uint32_t rotr(uint32_t x, int k) { return (x >> k) | (x << (32 - k)); }
void sha256_compress(const uint8_t* l, const uint8_t* r, uint8_t* out) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++) {
    const uint8_t* q = i < 8 ? l + 4 * i : r + 4 * (i - 8);
    w[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  for (int t = 16; t < 64; t++) {
    const uint32_t s0 = rotr(w[t - 15], 7) ^ rotr(w[t - 15], 18) ^ (w[t - 15] >> 3);
    const uint32_t s1 = rotr(w[t - 2], 17) ^ rotr(w[t - 2], 19) ^ (w[t - 2] >> 10);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint32_t a = iv[0], b = iv[1], c = iv[2], d = iv[3], e = iv[4], f = iv[5], g = iv[6], h = iv[7];
  for (int t = 0; t < 64; t++) {
    const uint32_t t1 = h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K256[t] + w[t];
    const uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
  }
  const uint32_t s[8] = {iv[0] + a, iv[1] + b, iv[2] + c, iv[3] + d, iv[4] + e, iv[5] + f, iv[6] + g, iv[7] + h};
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(s[i] >> (24 - 8 * k));
}

struct H {
  uint8_t b[32];
};
void combine(int kind, const H& l, const H& r, int depth, H* out) {
  if (kind == 0)
    sha256_compress(l.b, r.b, out->b);
  else
    pedersen_merkle(l.b, r.b, depth, out->b);
}

// ---- TreeState (tree_state.rs:193-264)
struct Tree {
  int kind, height;
  bool has_l = false, has_r = false, empty = true;
  H left, right;
  std::vector<int> has_p;
  std::vector<H> par;
  const std::vector<H>* E;
  bool append(const H& h) {
    if (!has_l) {
      left = h, has_l = true;
    } else if (!has_r) {
      right = h, has_r = true;
    } else {
      H fl = left, fr = right, comb;
      left = h;
      has_r = false;
      combine(kind, fl, fr, 0, &comb);
      for (int i = 0; i < height - 1; i++) {
        if (!has_p[i]) {
          par[i] = comb;
          has_p[i] = 1;
          return true;
        }
        H t;
        combine(kind, par[i], comb, i + 1, &t);
        comb = t;
        has_p[i] = 0;
      }
      return false;
    }
    empty = false;
    return true;
  }
  H root() const {
    if (empty) return (*E)[height];
    const H& l = has_l ? left : (*E)[0];
    const H& r = has_r ? right : (*E)[0];
    H root;
    combine(kind, l, r, 0, &root);
    for (int i = 0; i < height - 1; i++) {
      H t;
      if (has_p[i])
        combine(kind, par[i], root, i + 1, &t);
      else
        combine(kind, root, (*E)[i + 1], i + 1, &t);
      root = t;
    }
    return root;
  }
};

std::vector<H> g_empty[2];

const std::vector<H>& empties(int kind) {
  std::vector<H>& e = g_empty[kind];
  if (e.empty()) {
    H z;
    memset(z.b, 0, 32);
    if (kind == 1) z.b[0] = 1;
    e.push_back(z);
    for (int l = 0; l < 63; l++) {
      H t;
      combine(kind, e[l], e[l], l, &t);
      e.push_back(t);
    }
  }
  return e;
}

}  // namespace

extern "C" {

// gens: 3 x (x || y), canonical LE: find_group_hash(LE32(j), "Zcash_PH"), j = 0..2
int mc_init(const uint8_t* gens) {
  F one = {{1, 0, 0, 0}};
  ONE_M = to_mont(FR, one);
  // d = -10240 / 10241
  F a = {{10240, 0, 0, 0}}, b = {{10241, 0, 0, 0}};
  const F binv = inv_plain(FR, b);
  D_M = to_mont(FR, neg(FR, mul(FR, to_mont(FR, a), binv)));  // (10240 R)(1/10241) R^-1 = 10240/10241
  g_table.assign((size_t)3 * WINDOWS * 256, pt_zero());
  for (int g = 0; g < 3; g++) {
    P4 base = from_affine(gens + 64 * g);
    for (int w = 0; w < WINDOWS; w++) {
      P4* row = &g_table[((size_t)g * WINDOWS + w) * 256];
      row[0] = pt_zero();
      for (int i = 1; i < 256; i++) row[i] = pt_add(row[i - 1], base);
      for (int k = 0; k < 8; k++) base = pt_add(base, base);
    }
  }
  g_ready = true;
  empties(0);
  empties(1);
  return 0;
}

int mc_combine(int kind, const uint8_t* l, const uint8_t* r, int depth, uint8_t* out) {
  if (kind == 1 && !g_ready) return -1;
  H a, b, o;
  memcpy(a.b, l, 32);
  memcpy(b.b, r, 32);
  combine(kind, a, b, depth, &o);
  memcpy(out, o.b, 32);
  return 0;
}

// the reference's sequential path over a window: from the serialized state append the leaves,
// taking root() after marks[k] of them (marks sorted); returns 0, -1 bad state, -7 full tree
int mc_window(int kind, int height, const uint8_t* st, size_t st_len, size_t n, const uint8_t* leaves,
              size_t nm, const uint64_t* marks, uint8_t* roots) {
  if (kind == 1 && !g_ready) return -1;
  Tree t;
  t.kind = kind, t.height = height;
  t.has_p.assign(height - 1, 0);
  t.par.assign(height - 1, H());
  t.E = &empties(kind);
  size_t pos = 0;
  auto opt = [&](bool* has, H* h) {
    if (pos >= st_len) return false;
    *has = st[pos++] == 1;
    if (*has) {
      if (pos + 32 > st_len) return false;
      memcpy(h->b, st + pos, 32);
      pos += 32;
    }
    return true;
  };
  if (st_len) {
    bool ok = opt(&t.has_l, &t.left) && opt(&t.has_r, &t.right) && pos < st_len && st[pos] == height - 1;
    if (!ok) return -1;
    pos++;
    for (int i = 0; i < height - 1; i++) {
      bool h;
      if (!opt(&h, &t.par[i])) return -1;
      t.has_p[i] = h;
    }
    t.empty = !t.has_l && !t.has_r && std::none_of(t.has_p.begin(), t.has_p.end(), [](int x) { return x; });
  }
  size_t done = 0;
  for (size_t k = 0; k < nm; k++) {
    while (done < marks[k]) {
      H h;
      memcpy(h.b, leaves + 32 * done, 32);
      if (!t.append(h)) return -7;
      done++;
    }
    const H r = t.root();
    memcpy(roots + 32 * k, r.b, 32);
  }
  return 0;
}

}  // extern "C"
