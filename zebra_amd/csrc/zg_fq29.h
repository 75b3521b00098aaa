// zg_fq29.h -- Fq Montgomery products evaluated in 29-bit digits (generated: gen_fq29.py).
//
// Storage stays 12 x 32-bit words, Montgomery form R = 2^384 (zg_field.h). Only the products
// change representation: operands are split into 14 digits of 29 bits, so a digit product is
// < 2^58 and a whole column of up to 56 of them (a*b, a'*b' and m*p terms) fits one 64-bit
// accumulator. Each digit product is ONE v_mad_u64_u32 with no carry handling, against a
// v_mad_u64_u32 plus a v_addc_co_u32 per 32 x 32 product in the word form (zg_fips.h).
// The reduction divides by exactly 2^384 with mixed-radix digits (13 x 29 bits + 7 bits).
//
//   fq29_mul   a b             (392 digit products)
//   fq29_sqr   a^2             (105 + 196)
//   f2_mul29   Fq2 x y         schoolbook, two reductions (1,176)
//   f2_mul_fq29 (x0 s, x1 s)   (784)
//   f2_sqr29   Fq2 x^2         (x0 + x1)(x0 - x1), 2 x0 x1 (784)
//
// All functions are __host__ __device__: tests/native runs the identical code on the CPU.
#pragma once
#include "zg_field.h"
#include "zg_fq29_gen.h"
