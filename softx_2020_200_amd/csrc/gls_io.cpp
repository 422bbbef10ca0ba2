// gls_io.cpp — the drop-in I/O surface around the hot path, host C++:
//   * deal.II ParameterHandler text format (the subset Lethe's .prm files use):
//     `subsection` / `end` nesting, `set key = value`, `#` comments, `\` line continuation
//     (reference: source/core/parameters.cc, boundary_conditions.h:130-425 read through it);
//   * muParser-compatible expression compiler + evaluator for deal.II `Functions::ParsedFunction`
//     ("Function expression" with `;`-separated components, "Function constants" a=1, b=2,
//     variables x,y[,z],t; deal.II adds pi/Pi and the functions if/int/ceil/floor/cot/csc/sec/pow/
//     log(natural)/erfc to muParser's built-ins);
//   * VTU / PVTU / PVD writer with the reference's output fields (navier_stokes_base.cc:998-1086,
//     solutions_output.cc:14-59, post_processors.h:27-171): velocity, pressure, subdomain,
//     vorticity, q_criterion [, velocity_eulerian for SRF], one patch per cell with
//     `subdivision` intervals, Lagrange hexahedra / quadrilaterals when the velocity order > 1.
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/gls_native.h"

int gls_io_set_error(int code, const char *fmt, ...);  // gls_api.cpp (shared last-error buffer)

namespace {

std::string trim(const std::string &s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) ++a;
  while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}
// deal.II compares entry names after trimming and collapsing runs of blanks
std::string norm(const std::string &s) {
  std::string t = trim(s), o;
  bool sp = false;
  for (char ch : t) {
    if (std::isspace((unsigned char)ch)) {
      sp = true;
      continue;
    }
    if (sp && !o.empty()) o += ' ';
    sp = false;
    o += ch;
  }
  return o;
}

}  // namespace

// ============================================================================================
// Parameter files
// ============================================================================================
struct gls_prm {
  std::map<std::string, std::string> kv;  // "sub/sub/key" -> value
};

namespace {
int prm_parse(const std::string &text, gls_prm *p) {
  std::istringstream in(text);
  std::string raw, line;
  std::vector<std::string> path;
  int lineno = 0;
  while (std::getline(in, raw)) {
    ++lineno;
    // continuation: a trailing backslash joins the next line
    while (!raw.empty() && trim(raw).size() && trim(raw).back() == '\\') {
      std::string t = trim(raw);
      t.pop_back();
      std::string nxt;
      if (!std::getline(in, nxt)) break;
      ++lineno;
      raw = trim(t) + " " + trim(nxt);
    }
    const size_t hash = raw.find('#');
    line = trim(hash == std::string::npos ? raw : raw.substr(0, hash));
    if (line.empty()) continue;
    std::string w0 = line.substr(0, line.find_first_of(" \t"));
    if (w0 == "subsection") {
      path.push_back(norm(line.substr(10)));
    } else if (w0 == "end") {
      if (path.empty()) return gls_io_set_error(GLS_EIO, "prm line %d: 'end' without subsection", lineno);
      path.pop_back();
    } else if (w0 == "set") {
      const size_t eq = line.find('=');
      if (eq == std::string::npos) return gls_io_set_error(GLS_EIO, "prm line %d: 'set' without '='", lineno);
      std::string key;
      for (auto &s : path) key += s + "/";
      key += norm(line.substr(3, eq - 3));
      p->kv[key] = trim(line.substr(eq + 1));
    } else if (w0 == "include") {
      return gls_io_set_error(GLS_EIO, "prm line %d: 'include' is not supported", lineno);
    } else {
      return gls_io_set_error(GLS_EIO, "prm line %d: cannot parse '%s'", lineno, line.c_str());
    }
  }
  if (!path.empty()) return gls_io_set_error(GLS_EIO, "prm: subsection '%s' not closed", path.back().c_str());
  return GLS_OK;
}
}  // namespace

extern "C" {

int gls_prm_parse(const char *text, int is_path, gls_prm **out) {
  if (!text || !out) return gls_io_set_error(GLS_EINVAL, "gls_prm_parse: null argument");
  *out = nullptr;
  std::string body;
  if (is_path) {
    std::ifstream f(text);
    if (!f) return gls_io_set_error(GLS_EIO, "cannot open parameter file %s", text);
    std::stringstream ss;
    ss << f.rdbuf();
    body = ss.str();
  } else {
    body = text;
  }
  std::unique_ptr<gls_prm> p(new gls_prm);
  const int rc = prm_parse(body, p.get());
  if (rc != GLS_OK) return rc;
  *out = p.release();
  return GLS_OK;
}

// value of "subsection/.../key" (names normalised like deal.II); returns its length, copies
// min(len, cap-1) bytes + NUL into buf; GLS_ENOTFOUND when the entry is absent
int gls_prm_get(const gls_prm *p, const char *path, char *buf, int cap) {
  if (!p || !path) return gls_io_set_error(GLS_EINVAL, "gls_prm_get: null argument");
  std::string key;
  std::string s(path);
  size_t a = 0;
  while (true) {
    const size_t b = s.find('/', a);
    key += norm(s.substr(a, b == std::string::npos ? std::string::npos : b - a));
    if (b == std::string::npos) break;
    key += "/";
    a = b + 1;
  }
  auto it = p->kv.find(key);
  if (it == p->kv.end()) return GLS_ENOTFOUND;  // not an error: the caller applies the default
  const int n = (int)it->second.size();
  if (buf && cap > 0) {
    const int m = n < cap - 1 ? n : cap - 1;
    std::memcpy(buf, it->second.data(), (size_t)m);
    buf[m] = '\0';
  }
  return n;
}

int gls_prm_n_entries(const gls_prm *p) { return p ? (int)p->kv.size() : GLS_EINVAL; }

// i-th entry (sorted by path): path and value into the caller's buffers
int gls_prm_entry(const gls_prm *p, int i, char *path, int path_cap, char *value, int value_cap) {
  if (!p || i < 0 || i >= (int)p->kv.size()) return gls_io_set_error(GLS_EINVAL, "gls_prm_entry: index");
  auto it = p->kv.begin();
  std::advance(it, i);
  if (path && path_cap > 0) std::snprintf(path, (size_t)path_cap, "%s", it->first.c_str());
  if (value && value_cap > 0) std::snprintf(value, (size_t)value_cap, "%s", it->second.c_str());
  return GLS_OK;
}

void gls_prm_destroy(gls_prm *p) { delete p; }

}  // extern "C"

// ============================================================================================
// Expressions (muParser semantics as configured by deal.II's FunctionParser / ParsedFunction)
// ============================================================================================
namespace {

enum Op : int {
  PUSH_C, PUSH_V, NEG, ADD, SUB, MUL, DIV, POW, LT, GT, LE, GE, EQ, NE, AND, OR, NOT, SEL, F1, F2, FMIN, FMAX, FSUM
};
typedef double (*Fn1)(double);
typedef double (*Fn2)(double, double);

double f_sign(double x) { return (x > 0) - (x < 0); }
double f_rint(double x) { return std::rint(x); }
double f_int(double x) { return (double)(long long)std::lround(x); }  // deal.II mu_round
double f_cot(double x) { return 1.0 / std::tan(x); }
double f_csc(double x) { return 1.0 / std::sin(x); }
double f_sec(double x) { return 1.0 / std::cos(x); }
double f_log2(double x) { return std::log2(x); }

struct Fun1 { const char *name; Fn1 f; };
const Fun1 kFun1[] = {
    {"sin", std::sin},     {"cos", std::cos},     {"tan", std::tan},     {"asin", std::asin},  {"acos", std::acos},
    {"atan", std::atan},   {"sinh", std::sinh},   {"cosh", std::cosh},   {"tanh", std::tanh},  {"asinh", std::asinh},
    {"acosh", std::acosh}, {"atanh", std::atanh}, {"log2", f_log2},      {"log10", std::log10}, {"log", std::log},
    {"ln", std::log},      {"exp", std::exp},     {"sqrt", std::sqrt},   {"sign", f_sign},     {"rint", f_rint},
    {"abs", std::fabs},    {"int", f_int},        {"ceil", std::ceil},   {"floor", std::floor}, {"cot", f_cot},
    {"csc", f_csc},        {"sec", f_sec},        {"erfc", std::erfc},   {"erf", std::erf},
};
struct Fun2 { const char *name; Fn2 f; };
const Fun2 kFun2[] = {{"atan2", std::atan2}, {"pow", std::pow}, {"fmod", std::fmod}};

struct Instr {
  int op;
  double c;
  int i;  // var index / function index / arg count
};

struct Compiled {
  std::vector<Instr> code;
  int max_stack = 0;
};

class Parser {
 public:
  Parser(const std::string &s, const std::vector<std::string> &vars, const std::map<std::string, double> &consts)
      : s_(s), vars_(vars), consts_(consts) {}
  bool run(Compiled &out, std::string &err) {
    pos_ = 0;
    depth_ = 0;
    code_.clear();
    if (!ternary()) {
      err = err_;
      return false;
    }
    skip();
    if (pos_ != s_.size()) {
      err = "unexpected '" + s_.substr(pos_, 1) + "' at position " + std::to_string(pos_);
      return false;
    }
    out.code = code_;
    // stack depth
    int d = 0, mx = 0;
    for (auto &in : code_) {
      if (in.op == PUSH_C || in.op == PUSH_V) ++d;
      else if (in.op == NEG || in.op == NOT || in.op == F1) {
      } else if (in.op == SEL) d -= 2;
      else if (in.op == FMIN || in.op == FMAX || in.op == FSUM) d -= in.i - 1;
      else --d;
      mx = std::max(mx, d);
    }
    out.max_stack = mx;
    return true;
  }

 private:
  const std::string &s_;
  const std::vector<std::string> &vars_;
  const std::map<std::string, double> &consts_;
  size_t pos_ = 0;
  int depth_ = 0;
  std::vector<Instr> code_;
  std::string err_;

  void skip() {
    while (pos_ < s_.size() && std::isspace((unsigned char)s_[pos_])) ++pos_;
  }
  bool fail(const std::string &m) {
    if (err_.empty()) err_ = m + " at position " + std::to_string(pos_);
    return false;
  }
  bool eat(const char *tok) {
    skip();
    const size_t n = std::strlen(tok);
    if (s_.compare(pos_, n, tok) == 0) {
      // do not split '<=' into '<' '=' etc.
      if (n == 1 && (tok[0] == '<' || tok[0] == '>' || tok[0] == '!') && pos_ + 1 < s_.size() && s_[pos_ + 1] == '=')
        return false;
      if (n == 1 && (tok[0] == '&' || tok[0] == '|')) return false;
      pos_ += n;
      return true;
    }
    return false;
  }
  void emit(int op, double c = 0., int i = 0) { code_.push_back({op, c, i}); }

  // ternary: or ('?' ternary ':' ternary)?
  bool ternary() {
    if (++depth_ > 200) return fail("expression nested too deeply");
    if (!logic_or()) return false;
    if (eat("?")) {
      if (!ternary()) return false;
      if (!eat(":")) return fail("':' expected");
      if (!ternary()) return false;
      emit(SEL);
    }
    --depth_;
    return true;
  }
  bool logic_or() {
    if (!logic_and()) return false;
    while (eat("||")) {
      if (!logic_and()) return false;
      emit(OR);
    }
    return true;
  }
  bool logic_and() {
    if (!compare()) return false;
    while (eat("&&")) {
      if (!compare()) return false;
      emit(AND);
    }
    return true;
  }
  bool compare() {
    if (!additive()) return false;
    while (true) {
      int op = -1;
      if (eat("<=")) op = LE;
      else if (eat(">=")) op = GE;
      else if (eat("==")) op = EQ;
      else if (eat("!=")) op = NE;
      else if (eat("<")) op = LT;
      else if (eat(">")) op = GT;
      if (op < 0) return true;
      if (!additive()) return false;
      emit(op);
    }
  }
  bool additive() {
    if (!multiplicative()) return false;
    while (true) {
      if (eat("+")) {
        if (!multiplicative()) return false;
        emit(ADD);
      } else if (eat("-")) {
        if (!multiplicative()) return false;
        emit(SUB);
      } else {
        return true;
      }
    }
  }
  bool multiplicative() {
    if (!unary()) return false;
    while (true) {
      if (eat("*")) {
        if (!unary()) return false;
        emit(MUL);
      } else if (eat("/")) {
        if (!unary()) return false;
        emit(DIV);
      } else {
        return true;
      }
    }
  }
  // sign binds looser than '^' (-x^2 = -(x^2)); muParser documents the same for its sign operator
  bool unary() {
    if (eat("-")) {
      if (!unary()) return false;
      emit(NEG);
      return true;
    }
    if (eat("+")) return unary();
    if (eat("!")) {
      if (!unary()) return false;
      emit(NOT);
      return true;
    }
    return power();
  }
  bool power() {  // right associative
    if (!primary()) return false;
    if (eat("^")) {
      if (!unary()) return false;
      emit(POW);
    }
    return true;
  }
  bool primary() {
    skip();
    if (pos_ >= s_.size()) return fail("unexpected end of expression");
    const char ch = s_[pos_];
    if (std::isdigit((unsigned char)ch) || ch == '.') {
      const char *b = s_.c_str() + pos_;
      char *e = nullptr;
      const double v = std::strtod(b, &e);
      if (e == b) return fail("bad number");
      pos_ += (size_t)(e - b);
      emit(PUSH_C, v);
      return true;
    }
    if (std::isalpha((unsigned char)ch) || ch == '_') {
      size_t b = pos_;
      while (pos_ < s_.size() && (std::isalnum((unsigned char)s_[pos_]) || s_[pos_] == '_')) ++pos_;
      const std::string id = s_.substr(b, pos_ - b);
      skip();
      if (pos_ < s_.size() && s_[pos_] == '(') {
        ++pos_;
        int nargs = 0;
        skip();
        if (pos_ < s_.size() && s_[pos_] == ')') {
          ++pos_;
        } else {
          while (true) {
            if (!ternary()) return false;
            ++nargs;
            if (eat(",")) continue;
            if (eat(")")) break;
            return fail("',' or ')' expected in call of " + id);
          }
        }
        return call(id, nargs);
      }
      for (size_t i = 0; i < vars_.size(); ++i)
        if (vars_[i] == id) {
          emit(PUSH_V, 0., (int)i);
          return true;
        }
      auto it = consts_.find(id);
      if (it != consts_.end()) {
        emit(PUSH_C, it->second);
        return true;
      }
      return fail("unknown variable '" + id + "'");
    }
    if (ch == '(') {
      ++pos_;
      if (!ternary()) return false;
      if (!eat(")")) return fail("')' expected");
      return true;
    }
    return fail(std::string("unexpected '") + ch + "'");
  }
  bool call(const std::string &id, int nargs) {
    if (id == "if") {  // deal.II: if(condition, then, else)
      if (nargs != 3) return fail("if() takes 3 arguments");
      emit(SEL);
      return true;
    }
    if (id == "min" || id == "max" || id == "sum" || id == "avg") {
      if (nargs < 1) return fail(id + "() needs arguments");
      if (id == "avg") {
        emit(FSUM, 0., nargs);
        emit(PUSH_C, (double)nargs);
        emit(DIV);
      } else {
        emit(id == "min" ? FMIN : id == "max" ? FMAX : FSUM, 0., nargs);
      }
      return true;
    }
    for (size_t i = 0; i < sizeof(kFun1) / sizeof(kFun1[0]); ++i)
      if (id == kFun1[i].name) {
        if (nargs != 1) return fail(id + "() takes 1 argument");
        emit(F1, 0., (int)i);
        return true;
      }
    for (size_t i = 0; i < sizeof(kFun2) / sizeof(kFun2[0]); ++i)
      if (id == kFun2[i].name) {
        if (nargs != 2) return fail(id + "() takes 2 arguments");
        emit(F2, 0., (int)i);
        return true;
      }
    return fail("unknown function '" + id + "'");
  }
};

double run_code(const Compiled &c, const double *vars, double *stack) {
  int sp = 0;
  for (const Instr &in : c.code) {
    switch (in.op) {
      case PUSH_C: stack[sp++] = in.c; break;
      case PUSH_V: stack[sp++] = vars[in.i]; break;
      case NEG: stack[sp - 1] = -stack[sp - 1]; break;
      case NOT: stack[sp - 1] = stack[sp - 1] == 0.0 ? 1.0 : 0.0; break;
      case F1: stack[sp - 1] = kFun1[in.i].f(stack[sp - 1]); break;
      case F2: --sp; stack[sp - 1] = kFun2[in.i].f(stack[sp - 1], stack[sp]); break;
      case SEL: sp -= 2; stack[sp - 1] = stack[sp - 1] != 0.0 ? stack[sp] : stack[sp + 1]; break;
      case FMIN: case FMAX: case FSUM: {
        double r = stack[sp - in.i];
        for (int k = 1; k < in.i; ++k) {
          const double v = stack[sp - in.i + k];
          r = in.op == FMIN ? std::min(r, v) : in.op == FMAX ? std::max(r, v) : r + v;
        }
        sp -= in.i - 1;
        stack[sp - 1] = r;
        break;
      }
      default: {
        --sp;
        const double a = stack[sp - 1], b = stack[sp];
        double r = 0.;
        switch (in.op) {
          case ADD: r = a + b; break;
          case SUB: r = a - b; break;
          case MUL: r = a * b; break;
          case DIV: r = a / b; break;
          case POW: r = std::pow(a, b); break;
          case LT: r = a < b; break;
          case GT: r = a > b; break;
          case LE: r = a <= b; break;
          case GE: r = a >= b; break;
          case EQ: r = a == b; break;
          case NE: r = a != b; break;
          case AND: r = (a != 0.0) && (b != 0.0); break;
          case OR: r = (a != 0.0) || (b != 0.0); break;
        }
        stack[sp - 1] = r;
      }
    }
  }
  return stack[0];
}

std::vector<std::string> split(const std::string &s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (char ch : s) {
    if (ch == sep) {
      out.push_back(cur);
      cur.clear();
    } else {
      cur += ch;
    }
  }
  out.push_back(cur);
  return out;
}

}  // namespace

struct gls_expr {
  std::vector<std::string> vars;
  std::vector<Compiled> comps;
  int max_stack = 1;
};

extern "C" {

// expr: ';'-separated components (deal.II drops one trailing empty component, like
// Utilities::split_string_list); vars: comma-separated names ("x,y,z,t"); constants:
// "a=1, b=2" (may be NULL). pi and Pi are predefined (ParsedFunction), plus _pi and _e (muParser).
int gls_expr_create(const char *expr, const char *vars, const char *constants, gls_expr **out) {
  if (!expr || !vars || !out) return gls_io_set_error(GLS_EINVAL, "gls_expr_create: null argument");
  *out = nullptr;
  std::unique_ptr<gls_expr> e(new gls_expr);
  for (auto &v : split(vars, ',')) {
    const std::string t = trim(v);
    if (!t.empty()) e->vars.push_back(t);
  }
  std::map<std::string, double> consts = {{"pi", M_PI}, {"Pi", M_PI}, {"_pi", M_PI}, {"_e", M_E}};
  if (constants) {
    for (auto &kv : split(constants, ',')) {
      const std::string t = trim(kv);
      if (t.empty()) continue;
      const size_t eq = t.find('=');
      if (eq == std::string::npos) return gls_io_set_error(GLS_EINVAL, "constant '%s' without '='", t.c_str());
      const std::string name = trim(t.substr(0, eq)), val = trim(t.substr(eq + 1));
      char *end = nullptr;
      const double v = std::strtod(val.c_str(), &end);
      if (end == val.c_str() || trim(end).size())
        return gls_io_set_error(GLS_EINVAL, "constant '%s': '%s' is not a number", name.c_str(), val.c_str());
      consts[name] = v;
    }
  }
  std::vector<std::string> parts = split(expr, ';');
  if (parts.size() > 1 && trim(parts.back()).empty()) parts.pop_back();
  for (size_t c = 0; c < parts.size(); ++c) {
    const std::string t = trim(parts[c]);
    Compiled code;
    std::string err;
    Parser ps(t, e->vars, consts);
    if (t.empty() || !ps.run(code, err))
      return gls_io_set_error(GLS_EINVAL, "expression component %zu '%s': %s", c, t.c_str(),
                              t.empty() ? "empty" : err.c_str());
    e->max_stack = std::max(e->max_stack, code.max_stack);
    e->comps.push_back(std::move(code));
  }
  *out = e.release();
  return GLS_OK;
}

int gls_expr_n_components(const gls_expr *e) { return e ? (int)e->comps.size() : GLS_EINVAL; }

// out[p * n_comp + c] = component c at point p; values[p * n_vars + v] = variable v at point p
int gls_expr_eval(const gls_expr *e, int64_t n_points, const double *values, double *out) {
  if (!e || (n_points > 0 && (!out || (!values && !e->vars.empty()))))
    return gls_io_set_error(GLS_EINVAL, "gls_expr_eval: null argument");
  const int nv = (int)e->vars.size(), nc = (int)e->comps.size();
  std::vector<double> stack((size_t)e->max_stack + 4);
  for (int64_t p = 0; p < n_points; ++p)
    for (int c = 0; c < nc; ++c) out[p * nc + c] = run_code(e->comps[(size_t)c], values + p * nv, stack.data());
  return GLS_OK;
}

void gls_expr_destroy(gls_expr *e) { delete e; }

}  // extern "C"

// ============================================================================================
// VTU / PVTU / PVD output (DataOut::build_patches(mapping, subdivision) + write_vtu_and_pvd)
// ============================================================================================
namespace {

// 1D support points of FE_Q(k) on [0,1] (Gauss-Lobatto), as the kernels use
std::vector<double> lobatto_nodes(int k) {
  if (k == 1) return {0.0, 1.0};
  if (k == 2) return {0.0, 0.5, 1.0};
  const double a = 0.5 * (1.0 - 1.0 / std::sqrt(5.0));
  return {0.0, a, 1.0 - a, 1.0};  // k == 3
}
void lagrange(const std::vector<double> &xn, double x, double *v, double *d) {
  const int n = (int)xn.size();
  for (int a = 0; a < n; ++a) {
    double val = 1.0, der = 0.0;
    for (int b = 0; b < n; ++b) {
      if (b == a) continue;
      const double f = (x - xn[b]) / (xn[a] - xn[b]);
      der = der * f + val / (xn[a] - xn[b]);
      val *= f;
    }
    v[a] = val;
    d[a] = der;
  }
}

// VTK Lagrange hexahedron / quadrilateral point index of lattice point (i,j,k) of order n
// (vtkHigherOrderHexahedron::PointIndexFromIJK ordering: vertices, edges, faces, interior)
int vtk_lagrange_index(int dim, int n, int i, int j, int k) {
  const bool ib = i == 0 || i == n, jb = j == 0 || j == n, kb = dim == 2 || k == 0 || k == n;
  const int nb = (int)ib + (int)jb + (dim == 3 ? (int)kb : 0);
  if (dim == 2) {
    if (ib && jb) return i ? (j ? 2 : 1) : (j ? 3 : 0);
    int off = 4;
    if (!ib) return (i - 1) + (j ? 2 * (n - 1) : 0) + off;   // edges 0 (j=0), 2 (j=n)
    return (j - 1) + (i ? (n - 1) : 3 * (n - 1)) + off;      // edges 1 (i=n), 3 (i=0)
    // interior handled below
  }
  if (nb == 3) return (i ? (j ? 2 : 1) : (j ? 3 : 0)) + (k ? 4 : 0);
  int off = 8;
  if (nb == 2) {
    if (!ib) return (i - 1) + (j ? 2 * (n - 1) : 0) + (k ? 4 * (n - 1) : 0) + off;
    if (!jb) return (j - 1) + (i ? (n - 1) : 3 * (n - 1)) + (k ? 4 * (n - 1) : 0) + off;
    off += 8 * (n - 1);
    return (k - 1) + (n - 1) * (i ? (j ? 3 : 1) : (j ? 2 : 0)) + off;
  }
  off += 12 * (n - 1);
  const int f = (n - 1) * (n - 1);
  if (nb == 1) {
    if (ib) return (j - 1) + (n - 1) * (k - 1) + (i ? f : 0) + off;
    off += 2 * f;
    if (jb) return (i - 1) + (n - 1) * (k - 1) + (j ? f : 0) + off;
    off += 2 * f;
    return (i - 1) + (n - 1) * (j - 1) + (k ? f : 0) + off;
  }
  off += 6 * f;
  return off + (i - 1) + (n - 1) * ((j - 1) + (n - 1) * (k - 1));
}
int vtk_lagrange_index_2d_interior(int n, int i, int j) { return 4 * n + (i - 1) + (n - 1) * (j - 1); }

const char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
void base64(const unsigned char *p, size_t n, std::string &o) {
  size_t i = 0;
  for (; i + 2 < n; i += 3) {
    const unsigned v = (unsigned)p[i] << 16 | (unsigned)p[i + 1] << 8 | p[i + 2];
    o += kB64[v >> 18 & 63];
    o += kB64[v >> 12 & 63];
    o += kB64[v >> 6 & 63];
    o += kB64[v & 63];
  }
  if (i < n) {
    unsigned v = (unsigned)p[i] << 16;
    if (i + 1 < n) v |= (unsigned)p[i + 1] << 8;
    o += kB64[v >> 18 & 63];
    o += kB64[v >> 12 & 63];
    o += i + 1 < n ? kB64[v >> 6 & 63] : '=';
    o += '=';
  }
}
template <typename T>
void write_array(std::ostream &f, const char *type, const char *name, int ncomp, const std::vector<T> &a, bool binary) {
  f << "    <DataArray type=\"" << type << "\"";
  if (name) f << " Name=\"" << name << "\"";
  if (ncomp > 1) f << " NumberOfComponents=\"" << ncomp << "\"";
  f << " format=\"" << (binary ? "binary" : "ascii") << "\">\n";
  if (binary) {
    const uint64_t nb = a.size() * sizeof(T);
    std::vector<unsigned char> buf(sizeof(uint64_t) + nb);
    std::memcpy(buf.data(), &nb, sizeof(uint64_t));
    if (nb) std::memcpy(buf.data() + sizeof(uint64_t), a.data(), nb);
    std::string s;
    s.reserve(buf.size() * 4 / 3 + 8);
    base64(buf.data(), buf.size(), s);
    f << s << "\n";
  } else {
    f.precision(17);
    for (size_t i = 0; i < a.size(); ++i) f << a[i] << ((i + 1) % 12 ? " " : "\n");
    f << "\n";
  }
  f << "    </DataArray>\n";
}

}  // namespace

extern "C" {

// One VTU piece: a patch per cell with `subdivision` intervals per direction; point data
// velocity (3 comps), pressure, subdomain, vorticity, q_criterion [, velocity_eulerian if srf].
// solution: HOST vector in this library's layout. q_criterion reproduces the reference's
// QCriterionPostprocessor literally: its p1/r1 accumulators are declared outside the point loop
// (post_processors.h:84-115), so the value at patch point p is 0.5 * sum_{p'<=p} (|W|^2 - |S|^2).
int gls_vtu_write(const char *filename, const gls_mesh_desc *m, const double *sol, int subdivision, int subdomain,
                  int binary) {
  const bool mapped = m && m->map_degree > 0;
  if (!filename || !m || !sol || !m->cell_vnodes || (!m->cell_h && !(mapped && m->cell_support)))
    return gls_io_set_error(GLS_EINVAL, "gls_vtu_write: null argument");
  const int dim = m->dim, k = m->k, kp = m->kp, ns = subdivision > 0 ? subdivision : 1;
  if ((dim != 2 && dim != 3) || k < 1 || k > 3 || kp < 1 || kp > k)
    return gls_io_set_error(GLS_EINVAL, "gls_vtu_write: unsupported element");
  const int nk = k + 1, nkp = kp + 1, nvl = dim == 3 ? nk * nk * nk : nk * nk;
  const int npl = dim == 3 ? nkp * nkp * nkp : nkp * nkp;
  const int np1 = ns + 1, npp = dim == 3 ? np1 * np1 * np1 : np1 * np1;
  const bool high = k > 1;  // navier_stokes_base.cc:1027-1029 write_higher_order_cells
  const int64_t nc = m->n_cells;
  const std::vector<double> xv = lobatto_nodes(k), xp = lobatto_nodes(kp);
  // 1D tables at the patch points
  std::vector<double> Vv(np1 * nk), Dv(np1 * nk), Vp(np1 * nkp), Dp(np1 * nkp);
  for (int t = 0; t < np1; ++t) {
    lagrange(xv, (double)t / ns, &Vv[t * nk], &Dv[t * nk]);
    lagrange(xp, (double)t / ns, &Vp[t * nkp], &Dp[t * nkp]);
  }
  const int64_t npts = nc * npp;
  std::vector<double> pts((size_t)npts * 3), vel((size_t)npts * 3), pre((size_t)npts), vort((size_t)npts * (dim == 3 ? 3 : 1)),
      qcr((size_t)npts), sub((size_t)npts, (double)subdomain), eul;
  if (m->srf) eul.resize((size_t)npts * 3);
  const int64_t nvdof = (int64_t)dim * m->n_vnodes;
  // mapped cells: MappingQ(md) through the support points (build_patches(mapping, ...),
  // navier_stokes_base.cc:1062): patch point positions and J^-T for the gradients
  const int md = mapped ? m->map_degree : 1, nm = md + 1, nsup = dim == 3 ? nm * nm * nm : nm * nm;
  std::vector<double> Vm(np1 * nm), Dm(np1 * nm);
  if (mapped) {
    const std::vector<double> xm = lobatto_nodes(md);
    for (int t = 0; t < np1; ++t) lagrange(xm, (double)t / ns, &Vm[t * nm], &Dm[t * nm]);
  }
  const double one[3] = {1.0, 1.0, 1.0};
  for (int64_t c = 0; c < nc; ++c) {
    const int32_t *cv = m->cell_vnodes + c * nvl;
    const int32_t *cp = m->cell_pnodes ? m->cell_pnodes + c * npl : cv;
    const double *h = mapped ? one : m->cell_h + c * dim;
    double p1 = 0.0, r1 = 0.0;  // see the q_criterion note above
    for (int p = 0; p < npp; ++p) {
      const int t0 = p % np1, t1 = (p / np1) % np1, t2 = dim == 3 ? p / (np1 * np1) : 0;
      const int64_t P = c * npp + p;
      double x[3] = {0, 0, 0};
      const int tt[3] = {t0, t1, t2};
      double JI[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
      if (mapped) {
        double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
        const double *S = m->cell_support + c * nsup * dim;
        for (int b = 0; b < nsup; ++b) {
          const int b0i = b % nm, b1i = (b / nm) % nm, b2i = dim == 3 ? b / (nm * nm) : 0;
          const double v0 = Vm[t0 * nm + b0i], v1 = Vm[t1 * nm + b1i], v2 = dim == 3 ? Vm[t2 * nm + b2i] : 1.0;
          const double gr[3] = {Dm[t0 * nm + b0i] * v1 * v2, v0 * Dm[t1 * nm + b1i] * v2,
                                dim == 3 ? v0 * v1 * Dm[t2 * nm + b2i] : 0.0};
          for (int i = 0; i < dim; ++i) {
            x[i] += S[b * dim + i] * v0 * v1 * v2;
            for (int a = 0; a < dim; ++a) J[i][a] += S[b * dim + i] * gr[a];
          }
        }
        if (dim == 2) {
          const double det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
          JI[0][0] = J[1][1] / det; JI[0][1] = -J[0][1] / det; JI[1][0] = -J[1][0] / det; JI[1][1] = J[0][0] / det;
        } else {
          const double det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                             J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
          for (int a = 0; a < 3; ++a)
            for (int i = 0; i < 3; ++i)
              JI[a][i] = (J[(i + 1) % 3][(a + 1) % 3] * J[(i + 2) % 3][(a + 2) % 3] -
                          J[(i + 1) % 3][(a + 2) % 3] * J[(i + 2) % 3][(a + 1) % 3]) / det;
        }
      } else {
        for (int d = 0; d < dim; ++d) x[d] = (m->cell_x0 ? m->cell_x0[c * dim + d] : 0.0) + h[d] * tt[d] / ns;
      }
      double u[3] = {0, 0, 0}, G[3][3] = {{0}}, pv = 0.0;
      for (int a = 0; a < nvl; ++a) {
        const int a0 = a % nk, a1 = (a / nk) % nk, a2 = dim == 3 ? a / (nk * nk) : 0;
        const double b0 = Vv[t0 * nk + a0], b1 = Vv[t1 * nk + a1], b2 = dim == 3 ? Vv[t2 * nk + a2] : 1.0;
        const double gref[3] = {Dv[t0 * nk + a0] * b1 * b2 / h[0], b0 * Dv[t1 * nk + a1] * b2 / h[1],
                                dim == 3 ? b0 * b1 * Dv[t2 * nk + a2] / h[2] : 0.0};
        double g[3] = {gref[0], gref[1], gref[2]};
        if (mapped)
          for (int i = 0; i < dim; ++i) {
            g[i] = 0.0;
            for (int e = 0; e < dim; ++e) g[i] += JI[e][i] * gref[e];
          }
        const double phi = b0 * b1 * b2;
        for (int d = 0; d < dim; ++d) {
          const double ud = sol[(int64_t)cv[a] * dim + d];
          u[d] += ud * phi;
          for (int e = 0; e < dim; ++e) G[d][e] += ud * g[e];
        }
      }
      for (int a = 0; a < npl; ++a) {
        const int a0 = a % nkp, a1 = (a / nkp) % nkp, a2 = dim == 3 ? a / (nkp * nkp) : 0;
        pv += sol[nvdof + cp[a]] * Vp[t0 * nkp + a0] * Vp[t1 * nkp + a1] * (dim == 3 ? Vp[t2 * nkp + a2] : 1.0);
      }
      for (int d = 0; d < 3; ++d) {
        pts[3 * P + d] = x[d];
        vel[3 * P + d] = u[d];
      }
      pre[P] = pv;
      if (dim == 3) {  // post_processors.h:41-50
        vort[3 * P + 0] = G[2][1] - G[1][2];
        vort[3 * P + 1] = G[0][2] - G[2][0];
        vort[3 * P + 2] = G[1][0] - G[0][1];
      } else {
        vort[P] = G[1][0] - G[0][1];
      }
      for (int j = 0; j < dim; ++j)
        for (int e = 0; e < dim; ++e) {
          const double W = 0.5 * (G[j][e] - G[e][j]), S = 0.5 * (G[j][e] + G[e][j]);
          p1 += W * W;
          r1 += S * S;
        }
      qcr[P] = 0.5 * (p1 - r1);
      if (m->srf) {  // post_processors.h:138-160: u + Omega x x
        const double *o = m->omega;
        if (dim == 3) {
          eul[3 * P + 0] = u[0] + o[1] * x[2] - o[2] * x[1];
          eul[3 * P + 1] = u[1] + o[2] * x[0] - o[0] * x[2];
          eul[3 * P + 2] = u[2] + o[0] * x[1] - o[1] * x[0];
        } else {
          eul[3 * P + 0] = u[0] - o[2] * x[1];
          eul[3 * P + 1] = u[1] + o[2] * x[0];
          eul[3 * P + 2] = 0.0;
        }
      }
    }
  }
  // connectivity
  std::vector<int64_t> conn, offs;
  std::vector<uint8_t> types;
  if (high) {  // one Lagrange cell of order ns per patch
    std::vector<int> perm(npp);
    for (int p = 0; p < npp; ++p) {
      const int i = p % np1, j = (p / np1) % np1, kk = dim == 3 ? p / (np1 * np1) : 0;
      int idx;
      if (dim == 2 && i > 0 && i < ns && j > 0 && j < ns) idx = vtk_lagrange_index_2d_interior(ns, i, j);
      else idx = vtk_lagrange_index(dim, ns, i, j, kk);
      perm[idx] = p;
    }
    conn.reserve((size_t)(nc * npp));
    for (int64_t c = 0; c < nc; ++c) {
      for (int q = 0; q < npp; ++q) conn.push_back(c * npp + perm[q]);
      offs.push_back((c + 1) * npp);
      types.push_back(dim == 3 ? 72 : 70);  // VTK_LAGRANGE_HEXAHEDRON / _QUADRILATERAL
    }
  } else {  // ns^dim linear cells per patch
    const int nsub = dim == 3 ? ns * ns * ns : ns * ns, nv = dim == 3 ? 8 : 4;
    const int corner[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};
    for (int64_t c = 0; c < nc; ++c)
      for (int s = 0; s < nsub; ++s) {
        const int s0 = s % ns, s1 = (s / ns) % ns, s2 = dim == 3 ? s / (ns * ns) : 0;
        for (int v = 0; v < nv; ++v)
          conn.push_back(c * npp + (s0 + corner[v][0]) + np1 * ((s1 + corner[v][1]) + np1 * (s2 + corner[v][2])));
        offs.push_back((int64_t)conn.size());
        types.push_back(dim == 3 ? 12 : 9);  // VTK_HEXAHEDRON / VTK_QUAD
      }
  }
  std::ofstream f(filename, std::ios::binary);
  if (!f) return gls_io_set_error(GLS_EIO, "cannot write %s", filename);
  f << "<?xml version=\"1.0\"?>\n<VTKFile type=\"UnstructuredGrid\" version=\"1.0\" byte_order=\"LittleEndian\""
       " header_type=\"UInt64\">\n<UnstructuredGrid>\n<Piece NumberOfPoints=\""
    << npts << "\" NumberOfCells=\"" << types.size() << "\">\n  <Points>\n";
  write_array(f, "Float64", nullptr, 3, pts, binary);
  f << "  </Points>\n  <Cells>\n";
  write_array(f, "Int64", "connectivity", 1, conn, binary);
  write_array(f, "Int64", "offsets", 1, offs, binary);
  write_array(f, "UInt8", "types", 1, types, binary);
  f << "  </Cells>\n  <PointData Scalars=\"pressure\" Vectors=\"velocity\">\n";
  write_array(f, "Float64", "velocity", 3, vel, binary);
  write_array(f, "Float64", "pressure", 1, pre, binary);
  write_array(f, "Float64", "subdomain", 1, sub, binary);
  write_array(f, "Float64", "vorticity", dim == 3 ? 3 : 1, vort, binary);
  write_array(f, "Float64", "q_criterion", 1, qcr, binary);
  if (m->srf) write_array(f, "Float64", "velocity_eulerian", 3, eul, binary);
  f << "  </PointData>\n</Piece>\n</UnstructuredGrid>\n</VTKFile>\n";
  return f.good() ? GLS_OK : gls_io_set_error(GLS_EIO, "write error on %s", filename);
}

// parallel master record (write_pvtu_record) over the ranks' pieces
int gls_pvtu_write(const char *filename, int dim, int srf, int n_pieces, const char *const *pieces) {
  if (!filename || n_pieces < 0 || (n_pieces && !pieces)) return gls_io_set_error(GLS_EINVAL, "gls_pvtu_write");
  std::ofstream f(filename);
  if (!f) return gls_io_set_error(GLS_EIO, "cannot write %s", filename);
  f << "<?xml version=\"1.0\"?>\n<VTKFile type=\"PUnstructuredGrid\" version=\"1.0\" byte_order=\"LittleEndian\""
       " header_type=\"UInt64\">\n<PUnstructuredGrid GhostLevel=\"0\">\n  <PPoints>\n"
       "    <PDataArray type=\"Float64\" NumberOfComponents=\"3\"/>\n  </PPoints>\n"
       "  <PPointData Scalars=\"pressure\" Vectors=\"velocity\">\n"
       "    <PDataArray type=\"Float64\" Name=\"velocity\" NumberOfComponents=\"3\"/>\n"
       "    <PDataArray type=\"Float64\" Name=\"pressure\"/>\n"
       "    <PDataArray type=\"Float64\" Name=\"subdomain\"/>\n"
       "    <PDataArray type=\"Float64\" Name=\"vorticity\""
    << (dim == 3 ? " NumberOfComponents=\"3\"" : "") << "/>\n    <PDataArray type=\"Float64\" Name=\"q_criterion\"/>\n";
  if (srf) f << "    <PDataArray type=\"Float64\" Name=\"velocity_eulerian\" NumberOfComponents=\"3\"/>\n";
  f << "  </PPointData>\n";
  for (int i = 0; i < n_pieces; ++i) f << "  <Piece Source=\"" << pieces[i] << "\"/>\n";
  f << "</PUnstructuredGrid>\n</VTKFile>\n";
  return f.good() ? GLS_OK : gls_io_set_error(GLS_EIO, "write error on %s", filename);
}

// time series record (DataOutBase::write_pvd_record with PVDHandler's (time, file) list)
int gls_pvd_write(const char *filename, int n, const double *times, const char *const *files) {
  if (!filename || n < 0 || (n && (!times || !files))) return gls_io_set_error(GLS_EINVAL, "gls_pvd_write");
  std::ofstream f(filename);
  if (!f) return gls_io_set_error(GLS_EIO, "cannot write %s", filename);
  f.precision(17);
  f << "<?xml version=\"1.0\"?>\n<VTKFile type=\"Collection\" version=\"0.1\" ByteOrder=\"LittleEndian\">\n"
       "  <Collection>\n";
  for (int i = 0; i < n; ++i)
    f << "    <DataSet timestep=\"" << times[i] << "\" group=\"\" part=\"0\" file=\"" << files[i] << "\"/>\n";
  f << "  </Collection>\n</VTKFile>\n";
  return f.good() ? GLS_OK : gls_io_set_error(GLS_EIO, "write error on %s", filename);
}

}  // extern "C"
