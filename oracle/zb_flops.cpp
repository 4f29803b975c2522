/*
 * zb_flops.cpp — the oracle with counted arithmetic (TEST / MEASUREMENT INFRASTRUCTURE ONLY).
 *
 * SURVEY.md §8(d) asks for the algorithmic FLOPs per env-step from an instrumented build of the
 * CPU twin. This file compiles oracle/zb_oracle.c unchanged as C++ with `real` replaced by
 * CReal, a float whose every arithmetic operation increments a counter: +, -, *, / and the
 * compares of the physics, and the square roots and transcendental functions by name. The
 * float-typed glue around the physics (observation packing, RNG, actuator planner) is plain
 * float and is not counted: it is a few hundred operations per env-step against millions.
 * Results agree with liboracle_zbot.so to rounding (a mixed float / double expression is
 * evaluated in float here, in double there); the operation counts are the same. Read by
 * scripts/count_flops.py.
 */
#include <cmath>
#include <cstdint>
#include <type_traits>

namespace zbf {
struct Counts {
  uint64_t add, mul, div, sqrt, trans, cmp;
};
static Counts g;
}  // namespace zbf

struct CReal {
  float v;
  CReal() = default;
  CReal(float x) : v(x) {}
  CReal(double x) : v((float)x) {}
  CReal(int x) : v((float)x) {}
  CReal(unsigned x) : v((float)x) {}
  CReal(long x) : v((float)x) {}
  operator float() const { return v; }
  CReal& operator+=(CReal o) { zbf::g.add++; v += o.v; return *this; }
  CReal& operator-=(CReal o) { zbf::g.add++; v -= o.v; return *this; }
  CReal& operator*=(CReal o) { zbf::g.mul++; v *= o.v; return *this; }
  CReal& operator/=(CReal o) { zbf::g.div++; v /= o.v; return *this; }
  CReal operator-() const { return CReal(-v); }
  CReal operator+() const { return *this; }
};
template <class T>
using arith = std::enable_if_t<std::is_arithmetic_v<T>, int>;
#define ZBF_BIN(OP, CNT)                                                              \
  inline CReal operator OP(CReal a, CReal b) { zbf::g.CNT++; return CReal(a.v OP b.v); } \
  template <class T, arith<T> = 0>                                                   \
  inline CReal operator OP(CReal a, T b) { zbf::g.CNT++; return CReal(a.v OP (float)b); } \
  template <class T, arith<T> = 0>                                                   \
  inline CReal operator OP(T a, CReal b) { zbf::g.CNT++; return CReal((float)a OP b.v); }
ZBF_BIN(+, add)
ZBF_BIN(-, add)
ZBF_BIN(*, mul)
ZBF_BIN(/, div)
#define ZBF_CMP(OP)                                                                   \
  inline bool operator OP(CReal a, CReal b) { zbf::g.cmp++; return a.v OP b.v; }     \
  template <class T, arith<T> = 0>                                                   \
  inline bool operator OP(CReal a, T b) { zbf::g.cmp++; return a.v OP (float)b; }    \
  template <class T, arith<T> = 0>                                                   \
  inline bool operator OP(T a, CReal b) { zbf::g.cmp++; return (float)a OP b.v; }
ZBF_CMP(<)
ZBF_CMP(>)
ZBF_CMP(<=)
ZBF_CMP(>=)
ZBF_CMP(==)
ZBF_CMP(!=)

static inline CReal zbf_sqrt(CReal x) { zbf::g.sqrt++; return CReal(sqrtf(x.v)); }
static inline CReal zbf_t1(float (*f)(float), CReal x) { zbf::g.trans++; return CReal(f(x.v)); }
static inline CReal zbf_sin(CReal x) { return zbf_t1(sinf, x); }
static inline CReal zbf_cos(CReal x) { return zbf_t1(cosf, x); }
static inline CReal zbf_exp(CReal x) { return zbf_t1(expf, x); }
static inline CReal zbf_log(CReal x) { return zbf_t1(logf, x); }
static inline CReal zbf_fabs(CReal x) { return CReal(fabsf(x.v)); } /* a sign-bit operation */
static inline CReal zbf_asin(CReal x) { return zbf_t1(asinf, x); }
static inline CReal zbf_pow(CReal x, CReal y) { zbf::g.trans++; return CReal(powf(x.v, y.v)); }
static inline CReal zbf_atan2(CReal y, CReal x) { zbf::g.trans++; return CReal(atan2f(y.v, x.v)); }

typedef CReal real;
#define SQRT zbf_sqrt
#define SIN zbf_sin
#define COS zbf_cos
#define EXP zbf_exp
#define LOG zbf_log
#define POW zbf_pow
#define FABS zbf_fabs
#define ATAN2 zbf_atan2
#define ASIN zbf_asin
#define ZBO_COUNT 1

#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
extern "C" {
#include "zb_oracle.c"
}

extern "C" {
/* counts since the last reset: add (incl. subtract), mul, div, sqrt, transcendental, compare */
void zbo_flops_get(uint64_t out[6]) {
  out[0] = zbf::g.add;
  out[1] = zbf::g.mul;
  out[2] = zbf::g.div;
  out[3] = zbf::g.sqrt;
  out[4] = zbf::g.trans;
  out[5] = zbf::g.cmp;
}
void zbo_flops_reset(void) { zbf::g = zbf::Counts{}; }
}
