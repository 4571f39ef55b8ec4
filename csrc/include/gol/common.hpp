// gol-mi355x: common types, error handling and the bit-sliced B3/S23 rule.
//
// The reference keeps one ASCII byte per cell and evaluates B3/S23 with
// nested branchy loops (serial: src/game.c:60-101; MPI ASCII-sum form:
// src/game_mpi.c:61-87; CUDA 1 thread/cell: src/game_cuda.cu:128-148).
// This framework evaluates the rule on 32 cells at once with bit-sliced
// adders, written so that every step maps onto one CDNA4 VALU instruction
// (v_bitop3_b32 / v_alignbit_b32 / DPP moves).  The host versions below are
// bit-exact emulations used by the CPU backend and the test oracles.
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

// Functions shared by host code and HIP kernels (e.g. the RNG) carry GOL_HD.
#if defined(__HIP__)
#define GOL_HD __host__ __device__
#else
#define GOL_HD
#endif

namespace gol {

enum class Layout : int { U8 = 0, Bits = 1 };

inline const char* layout_name(Layout l) { return l == Layout::Bits ? "bits" : "u8"; }

// Fail-stop error (the reference calls perror_exit / cudaSafeCall and exits:
// src/game.c:19-23, src/game_cuda.cu:18-27).  We throw so that Python callers
// get a RuntimeError; the CLI catches, prints and exits non-zero.
struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] void fail(const std::string& msg);

#define GOL_REQUIRE(cond, msg)                                                  \
  do {                                                                          \
    if (!(cond)) ::gol::fail(std::string(__FILE__) + ":" +                      \
                             std::to_string(__LINE__) + ": " + (msg));         \
  } while (0)

constexpr int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
constexpr int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// ---------------------------------------------------------------------------
// v_bitop3_b32 truth tables.  Operand k of bitop3(a, b, c) contributes the
// 8-bit pattern {0xF0, 0xCC, 0xAA}[k]; the immediate is the function applied
// to those patterns (same convention as LLVM's BitOp3 lowering).
// ---------------------------------------------------------------------------
namespace tt {
constexpr uint8_t A = 0xF0, B = 0xCC, C = 0xAA;
constexpr uint8_t XOR3 = A ^ B ^ C;                      // parity
constexpr uint8_t MAJ = (A & B) | (A & C) | (B & C);     // carry
constexpr uint8_t ANDN_XOR = uint8_t(~A & (B ^ C));      // ~a & (b ^ c)
constexpr uint8_t EQ_NE = uint8_t(~(A ^ B) & (A ^ C));   // (a == b) & (a != c)
constexpr uint8_t SEL = uint8_t((A & B) | (~A & C));     // a ? b : c
constexpr uint8_t OR_XOR = uint8_t(A | (B ^ C));         // a | (b ^ c)
constexpr uint8_t AND3 = A & B & C;
}  // namespace tt

// Host emulation of v_bitop3_b32 (bit-exact): each result bit is
// TT[(a<<2)|(b<<1)|c].
template <unsigned TT>
inline uint32_t bop3_host(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r = 0;
  if (TT & 0x01) r |= ~a & ~b & ~c;
  if (TT & 0x02) r |= ~a & ~b & c;
  if (TT & 0x04) r |= ~a & b & ~c;
  if (TT & 0x08) r |= ~a & b & c;
  if (TT & 0x10) r |= a & ~b & ~c;
  if (TT & 0x20) r |= a & ~b & c;
  if (TT & 0x40) r |= a & b & ~c;
  if (TT & 0x80) r |= a & b & c;
  return r;
}

// Funnel shift: low 32 bits of ((hi:lo) >> s), s in [0,31]  (v_alignbit_b32).
inline uint32_t alignbit_host(uint32_t hi, uint32_t lo, unsigned s) {
  return uint32_t(((uint64_t(hi) << 32) | lo) >> s);
}

// Bit order: bit j of word w holds cell x = 32*w + j (LSB = leftmost cell).
// Horizontal 3-sum of a row: (h1,h0) = L + C + R as a 2-bit number.
struct HSum {
  uint32_t h0, h1;
};

inline HSum hsum_host(uint32_t left_word, uint32_t c, uint32_t right_word) {
  uint32_t l = alignbit_host(c, left_word, 31);   // cell x-1 at bit of x
  uint32_t r = alignbit_host(right_word, c, 1);   // cell x+1 at bit of x
  return {bop3_host<tt::XOR3>(l, c, r), bop3_host<tt::MAJ>(l, c, r)};
}

// B3/S23 from three horizontal sums (rows above, centre, below) and the centre
// cells.  S = 3x3 sum including the centre = x0 + 2*(x1 + y0) + 4*y1;
// next = (S == 3) | (C & S == 4).
inline uint32_t rule_host(HSum a, HSum b, HSum c, uint32_t ctr) {
  uint32_t x0 = bop3_host<tt::XOR3>(a.h0, b.h0, c.h0);
  uint32_t x1 = bop3_host<tt::MAJ>(a.h0, b.h0, c.h0);
  uint32_t y0 = bop3_host<tt::XOR3>(a.h1, b.h1, c.h1);
  uint32_t y1 = bop3_host<tt::MAJ>(a.h1, b.h1, c.h1);
  uint32_t s3 = bop3_host<tt::ANDN_XOR>(y1, x1, y0);  // x0=1: S==3
  uint32_t s4 = bop3_host<tt::EQ_NE>(x1, y0, y1);     // x0=0: S==4
  return bop3_host<tt::SEL>(x0, s3, ctr & s4);
}

}  // namespace gol
