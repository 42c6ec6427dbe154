// bandmath.hip -- band-math on merged canvases (processor/tile_merger.go:
// 523-731).
//
// The reference evaluates each ConfigPayLoad band expression with a fork of
// govaluate (github.com/edisonguo/govaluate, absent from /root/reference)
// over the namespaces' canvases converted to float32, then writes a Float32
// raster: pixels where any of the expression's variables equals its canvas
// nodata, and non-finite results, become the first namespace's nodata; a
// constant expression fills every valid pixel (tile_merger.go:663-724).
//
// Here the expression is compiled on the host (recursive descent) to a short
// postfix program that travels as a kernel argument; one thread evaluates a
// pixel from a register stack, reading each variable straight from its typed
// canvas (no float32 copies of the canvases).  Arithmetic is float32 per
// element with constants rounded to float32 -- the semantics the oracle
// restates; parity with the govaluate fork itself is unpinned.
// Grammar: ?: (right assoc.), ||, &&, == !=, < <= > >=, + -, * / %, ** (right
// assoc.), unary - ! +, numbers, variables, parentheses; comparisons and
// logic yield 1.0 / 0.0.
#include <hip/hip_runtime.h>

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/gskyhip.h"
#include "gsky_device.h"

namespace gsky {
namespace {

enum Op : int32_t {
  OP_VAR = 1, OP_CONST, OP_ADD, OP_SUB, OP_MUL, OP_DIV, OP_MOD, OP_POW, OP_NEG, OP_NOT,
  OP_LT, OP_LE, OP_GT, OP_GE, OP_EQ, OP_NE, OP_AND, OP_OR, OP_SEL
};

constexpr int kMaxCode = 96;
constexpr int kMaxStack = 16;
constexpr int kMaxVars = GSKYHIP_BANDMATH_MAX_VARS;

struct Prog {
  int32_t op[kMaxCode];
  float arg[kMaxCode];      // OP_VAR: variable index; OP_CONST: value
  int32_t n;
};

struct Vars {
  const void *data[kMaxVars];
  int32_t dtype[kMaxVars];
  double nodata[kMaxVars];
  int32_t used[kMaxVars];   // the variable's nodata masks the pixel
  int32_t n;
};

// ---------------------------------------------------------------- compiler
struct Parser {
  const char *s;
  const char *const *names;
  int n_names;
  Prog *p;
  int depth = 0, max_depth = 0;
  int err = 0;
  int used[kMaxVars] = {0};

  void ws() { while (*s && std::isspace((unsigned char)*s)) s++; }
  bool emit(int32_t op, float a, int delta) {
    if (p->n >= kMaxCode) { err = GSKYHIP_E_ARG; return false; }
    p->op[p->n] = op;
    p->arg[p->n] = a;
    p->n++;
    depth += delta;
    if (depth > max_depth) max_depth = depth;
    if (max_depth > kMaxStack) err = GSKYHIP_E_ARG;
    return true;
  }
  bool eat(const char *t) {
    ws();
    const size_t k = std::strlen(t);
    if (std::strncmp(s, t, k) == 0) { s += k; return true; }
    return false;
  }
  // ternary: or ( '?' ternary ':' ternary )?
  void ternary() {
    logic_or();
    if (err) return;
    if (eat("?")) {
      ternary();
      if (err) return;
      if (!eat(":")) { err = GSKYHIP_E_ARG; return; }
      ternary();
      emit(OP_SEL, 0, -2);
    }
  }
  void logic_or() {
    logic_and();
    while (!err && eat("||")) { logic_and(); emit(OP_OR, 0, -1); }
  }
  void logic_and() {
    equality();
    while (!err && eat("&&")) { equality(); emit(OP_AND, 0, -1); }
  }
  void equality() {
    relation();
    for (;;) {
      if (err) return;
      if (eat("==")) { relation(); emit(OP_EQ, 0, -1); }
      else if (eat("!=")) { relation(); emit(OP_NE, 0, -1); }
      else return;
    }
  }
  void relation() {
    additive();
    for (;;) {
      if (err) return;
      if (eat("<=")) { additive(); emit(OP_LE, 0, -1); }
      else if (eat(">=")) { additive(); emit(OP_GE, 0, -1); }
      else if (eat("<")) { additive(); emit(OP_LT, 0, -1); }
      else if (eat(">")) { additive(); emit(OP_GT, 0, -1); }
      else return;
    }
  }
  void additive() {
    multiplicative();
    for (;;) {
      if (err) return;
      if (eat("+")) { multiplicative(); emit(OP_ADD, 0, -1); }
      else if (eat("-")) { multiplicative(); emit(OP_SUB, 0, -1); }
      else return;
    }
  }
  void multiplicative() {
    power();
    for (;;) {
      if (err) return;
      ws();
      if (s[0] == '*' && s[1] != '*') { s++; power(); emit(OP_MUL, 0, -1); }
      else if (eat("/")) { power(); emit(OP_DIV, 0, -1); }
      else if (eat("%")) { power(); emit(OP_MOD, 0, -1); }
      else return;
    }
  }
  void power() {
    unary();
    if (!err && eat("**")) { power(); emit(OP_POW, 0, -1); }
  }
  void unary() {
    if (eat("-")) { unary(); emit(OP_NEG, 0, 0); return; }
    if (eat("+")) { unary(); return; }
    ws();
    if (s[0] == '!' && s[1] != '=') { s++; unary(); emit(OP_NOT, 0, 0); return; }
    primary();
  }
  void primary() {
    ws();
    if (eat("(")) {
      ternary();
      if (!err && !eat(")")) err = GSKYHIP_E_ARG;
      return;
    }
    if (std::isdigit((unsigned char)*s) || (*s == '.' && std::isdigit((unsigned char)s[1]))) {
      char *end = nullptr;
      const double v = std::strtod(s, &end);
      s = end;
      emit(OP_CONST, (float)v, 1);
      return;
    }
    if (std::isalpha((unsigned char)*s) || *s == '_') {
      const char *b = s;
      while (std::isalnum((unsigned char)*s) || *s == '_' || *s == '.') s++;
      const std::string id(b, s);
      for (int i = 0; i < n_names; i++) {
        if (names[i] && id == names[i]) {
          used[i] = 1;
          emit(OP_VAR, (float)i, 1);
          return;
        }
      }
      err = GSKYHIP_E_ARG;   // govaluate: "No parameter '<id>' found."
      return;
    }
    err = GSKYHIP_E_ARG;
  }
};

// ---------------------------------------------------------------- evaluation
__device__ __forceinline__ float load_as_f32(const void *d, int dtype, int64_t i, double &as64) {
  float v;
  switch (dtype) {
    case GSKYHIP_BYTE: v = (float)((const uint8_t *)d)[i]; break;
    case GSKYHIP_SIGNEDBYTE: v = (float)((const int8_t *)d)[i]; break;
    case GSKYHIP_INT16: v = (float)((const int16_t *)d)[i]; break;
    case GSKYHIP_UINT16: v = (float)((const uint16_t *)d)[i]; break;
    default: v = ((const float *)d)[i]; break;
  }
  as64 = (double)v;
  return v;
}

__global__ __launch_bounds__(256) void band_math_kernel(Prog prog, Vars vars, int64_t n_px, float out_nodata,
                                                        int scalar, float *__restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_px; i += (int64_t)gridDim.x * blockDim.x) {
    // tile_merger.go:664-677: a pixel is valid unless one of the variables is its nodata
    float x[kMaxVars];
    bool valid = true;
    for (int k = 0; k < vars.n; k++) {
      double d;
      x[k] = load_as_f32(vars.data[k], vars.dtype[k], i, d);
      if (vars.used[k] && d == vars.nodata[k]) valid = false;
    }
    if (!valid) { out[i] = out_nodata; continue; }
    float st[kMaxStack];
    int sp = 0;
    for (int c = 0; c < prog.n; c++) {
      const int op = prog.op[c];
      if (op == OP_VAR) { st[sp++] = x[(int)prog.arg[c]]; continue; }
      if (op == OP_CONST) { st[sp++] = prog.arg[c]; continue; }
      if (op == OP_NEG) { st[sp - 1] = -st[sp - 1]; continue; }
      if (op == OP_NOT) { st[sp - 1] = st[sp - 1] == 0.f ? 1.f : 0.f; continue; }
      if (op == OP_SEL) {
        const float b = st[--sp], a = st[--sp], cnd = st[sp - 1];
        st[sp - 1] = cnd != 0.f ? a : b;
        continue;
      }
      const float b = st[--sp], a = st[sp - 1];
      float r;
      switch (op) {
        case OP_ADD: r = a + b; break;
        case OP_SUB: r = a - b; break;
        case OP_MUL: r = a * b; break;
        case OP_DIV: r = a / b; break;
        case OP_MOD: r = fmodf(a, b); break;
        case OP_POW: r = powf(a, b); break;
        case OP_LT: r = a < b ? 1.f : 0.f; break;
        case OP_LE: r = a <= b ? 1.f : 0.f; break;
        case OP_GT: r = a > b ? 1.f : 0.f; break;
        case OP_GE: r = a >= b ? 1.f : 0.f; break;
        case OP_EQ: r = a == b ? 1.f : 0.f; break;
        case OP_NE: r = a != b ? 1.f : 0.f; break;
        case OP_AND: r = (a != 0.f && b != 0.f) ? 1.f : 0.f; break;
        default: r = (a != 0.f || b != 0.f) ? 1.f : 0.f; break;   // OP_OR
      }
      st[sp - 1] = r;
    }
    const float res = st[0];
    // tile_merger.go:698-722: a constant expression fills every valid pixel;
    // an array result drops non-finite values
    out[i] = (scalar || isfinite(res)) ? res : out_nodata;
  }
}

}  // namespace
}  // namespace gsky

using namespace gsky;

extern "C" int gskyhip_band_math(const char *expr, const char *const *var_names, const void *const *canvases,
                                 const int32_t *dtypes, const double *nodatas, int n_vars, int64_t n_px,
                                 double out_nodata, float *out, void *stream) {
  if (!expr || n_vars < 0 || n_vars > kMaxVars || n_px < 0 || (n_px > 0 && !out)) return GSKYHIP_E_ARG;
  Prog prog;
  std::memset(&prog, 0, sizeof(prog));
  Parser ps;
  ps.s = expr;
  ps.names = var_names;
  ps.n_names = n_vars;
  ps.p = &prog;
  ps.ternary();
  ps.ws();
  if (ps.err || *ps.s || prog.n == 0) return GSKYHIP_E_ARG;
  Vars vars;
  std::memset(&vars, 0, sizeof(vars));
  vars.n = n_vars;
  bool any = false;
  for (int k = 0; k < n_vars; k++) {
    if (!canvases || !dtypes || !nodatas || !canvases[k]) return GSKYHIP_E_ARG;
    switch (dtypes[k]) {
      case GSKYHIP_BYTE: case GSKYHIP_SIGNEDBYTE: case GSKYHIP_INT16: case GSKYHIP_UINT16: case GSKYHIP_FLOAT32:
        break;
      default: return GSKYHIP_E_TYPE;   // "raster type %s not recognised" (tile_merger.go:648-650)
    }
    vars.data[k] = canvases[k];
    vars.dtype[k] = dtypes[k];
    vars.nodata[k] = nodatas[k];
    vars.used[k] = 1;   // every variable of the axis masks the pixel, used or not (tile_merger.go:670-677)
    any = any || ps.used[k];
  }
  if (n_px == 0) return 0;
  const int64_t blocks = std::min<int64_t>((n_px + 255) / 256, 65536);
  hipLaunchKernelGGL(band_math_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, prog, vars, n_px,
                     (float)out_nodata, any ? 0 : 1, out);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}
