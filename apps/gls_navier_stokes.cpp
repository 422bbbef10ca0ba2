// gls_navier_stokes — parameter-file driven GLS Navier–Stokes application on MI355X: the drop-in
// for the reference's applications/gls_navier_stokes_{2d,3d} (the GLSNavierStokesSolver::solve
// flow, gls_navier_stokes.cc:1395-1423), built only on the C-ABI of libgls_native.so:
//   read prm (gls_prm_*) -> hyper_cube mesh + boundary conditions (setup_dofs :55-228) ->
//   initial condition (nodal | L2projection | viscous, :784-827) -> time loop (integrate, first
//   step with the BDF start-up, SDIRK stages; navier_stokes_base.cc:426-590) with the device
//   Newton/GMRES (gls_newton_solve) -> post-processing (L2 error vs the analytical solution,
//   enstrophy, kinetic energy, CFL; VTU/PVTU/PVD output).
// Results are printed as `key = value` lines and a final error table (own format); the numbers
// are what the parity tests compare with the reference's outputs.
//
// Usage: gls_navier_stokes [--dim 2|3] [--precond mg|jacobi] file.prm
// Scope: mesh type dealii / grid type hyper_cube (+ initial refinement; steady "number mesh adapt"
// with mesh adaptation type uniform, or kelly = Kelly-driven refinement and coarsening on a forest
// with hanging nodes, any number of levels); bc types noslip, function, periodic, slip.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <map>
#include <unordered_map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../include/gls_native.h"

namespace {

std::atomic<int> *g_abort = nullptr;  // --np: raised by a failing rank, every other rank stops
[[noreturn]] void die(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::fprintf(stderr, "gls_navier_stokes: ");
  std::vfprintf(stderr, fmt, ap);
  std::fprintf(stderr, "\n");
  va_end(ap);
  if (g_abort) g_abort->store(1);
  std::exit(1);
}
void ck(int rc, const char *what) {
  if (rc < 0 && rc != GLS_ENOCONV) die("%s failed (%d): %s", what, rc, gls_last_error());
}
void hk(hipError_t e, const char *what) {
  if (e != hipSuccess) die("%s: %s", what, hipGetErrorString(e));
}
std::string trim(const std::string &s) {
  const size_t a = s.find_first_not_of(" \t"), b = s.find_last_not_of(" \t");
  return a == std::string::npos ? "" : s.substr(a, b - a + 1);
}

// ---------------------------------------------------------------------------------------------
// parameters: entry names / defaults follow the reference's declarations
// (source/core/parameters.cc, include/core/boundary_conditions.h:130-330)
// ---------------------------------------------------------------------------------------------
struct Prm {
  gls_prm *h = nullptr;
  explicit Prm(const char *path) { ck(gls_prm_parse(path, 1, &h), "reading the parameter file"); }
  ~Prm() { gls_prm_destroy(h); }
  std::string get(const std::string &path, const std::string &dflt) const {
    const int n = gls_prm_get(h, path.c_str(), nullptr, 0);
    if (n == GLS_ENOTFOUND) return dflt;
    ck(n, "gls_prm_get");
    std::vector<char> buf((size_t)n + 1);
    gls_prm_get(h, path.c_str(), buf.data(), n + 1);
    return std::string(buf.data());
  }
  double d(const std::string &p, double dflt) const {
    const std::string s = get(p, "");
    if (s.empty()) return dflt;
    char *e = nullptr;
    const double v = std::strtod(s.c_str(), &e);
    if (e == s.c_str()) die("%s = '%s' is not a number", p.c_str(), s.c_str());
    return v;
  }
  int i(const std::string &p, int dflt) const { return (int)std::lround(d(p, dflt)); }
  bool b(const std::string &p, bool dflt) const {
    const std::string s = get(p, dflt ? "true" : "false");
    if (s == "true" || s == "yes") return true;
    if (s == "false" || s == "no") return false;
    die("%s = '%s' is not a bool", p.c_str(), s.c_str());
  }
};

// a ParsedFunction-style function read from subsection `sec`
struct Function {
  gls_expr *e = nullptr;
  int nc = 0;
  Function() = default;
  Function(const Prm &p, const std::string &sec, int dim, const std::string &dflt_expr) {
    const std::string vars = p.get(sec + "/Variable names", dim == 3 ? "x,y,z,t" : "x,y,t");
    const std::string ex = p.get(sec + "/Function expression", dflt_expr);
    const std::string cs = p.get(sec + "/Function constants", "");
    ck(gls_expr_create(ex.c_str(), vars.c_str(), cs.c_str(), &e), (sec + "/Function expression").c_str());
    nc = gls_expr_n_components(e);
    if (std::count(vars.begin(), vars.end(), ',') != dim) die("%s: expected %d variables", sec.c_str(), dim + 1);
  }
  Function(const Function &) = delete;
  Function &operator=(const Function &) = delete;
  Function(Function &&o) noexcept : e(o.e), nc(o.nc) { o.e = nullptr; }
  Function &operator=(Function &&o) noexcept {
    std::swap(e, o.e);
    nc = o.nc;
    return *this;
  }
  ~Function() { gls_expr_destroy(e); }
  // out[p*nc + c] at the points X[p*dim + d] and time t
  void eval(const std::vector<double> &X, int dim, double t, std::vector<double> &out) const {
    const int64_t n = (int64_t)X.size() / dim;
    std::vector<double> v((size_t)n * (dim + 1));
    for (int64_t q = 0; q < n; ++q) {
      for (int d = 0; d < dim; ++d) v[(size_t)(q * (dim + 1) + d)] = X[(size_t)(q * dim + d)];
      v[(size_t)(q * (dim + 1) + dim)] = t;
    }
    out.resize((size_t)n * nc);
    ck(gls_expr_eval(e, n, v.data(), out.data()), "gls_expr_eval");
  }
};

enum class Method { steady, bdf1, bdf2, bdf3, sdirk2, sdirk3 };

struct BC {
  std::string type;
  int id = 0, periodic_id = 1, periodic_direction = 0;
  Function f[3];
};

struct Params {
  int dim = 3;
  Method method = Method::steady;
  double dt = 1.0, t_end = 1.0, startup = 0.4;
  int mesh_adapt = 0, output_frequency = 1, subdivision = 1, log_frequency = 1;
  int adapt_frequency = 1;  // mesh adaptation/frequency (refine_mesh: step % frequency == 0)
  std::string output_path = "./", output_name = "out";
  double nu = 1.0;
  int k = 1, kp = 1;
  double lo = -1, hi = 1;
  bool colorize = false;
  int refinement = 0;
  // general meshes (gls_umesh): mesh type gmsh or a non-hyper_cube deal.II grid
  bool general = false;
  std::string mesh_type = "dealii", grid_type = "hyper_cube", grid_args = "-1 : 1 : false", mesh_file;
  bool qmapping_all = false;
  struct ManifoldPrm { int id = 0; std::string type = "none"; double arg[3] = {0, 0, 0}; };
  std::vector<ManifoldPrm> manifolds;
  int display_precision = 4, residual_precision = 4;
  std::vector<BC> bcs;
  bool source = false;
  Function force;
  std::string ic_type = "nodal";
  Function ic;
  double ic_nu = 1.0;
  bool analytical = false, analytical_verbose = false;
  std::string analytical_file = "L2Error";
  Function exact;
  bool enstrophy = false, kinetic = false, pp_verbose = false;
  double newton_tol = 1e-6;
  int newton_max = 10, newton_verbose = 0, lin_max = 1000, restart = 30;
  int nl_solver = GLS_NEWTON, skip_iterations = 1;  // non-linear solver/solver, skip iterations
  double lin_rel = 1e-3, lin_min = 1e-8;
  double ilu_atol = 1e-8, ilu_rtol = 1.0;
  int ilu_fill = 0;
  int lin_method = 0;  // linear solver/method: 0 gmres, 1 bicgstab, 2 amg
  int amg_ilu_fill = 0, amg_n_cycles = 1, amg_sweeps = 2, amg_overlap = 1;
  double amg_ilu_atol = 1e-12, amg_ilu_rtol = 1.0, amg_threshold = 1e-14;
  bool amg_w_cycles = false;
  std::string timer = "none";  // timer/type none | iteration | end (parameters.cc:136-164)
  bool srf = false;
  double omega[3] = {0, 0, 0};
  // mesh adaptation (parameters.cc:649-731): uniform, or kelly = one Kelly-driven refinement
  std::string madapt = "none";
  int kelly_variable = 0;  // 0 velocity, 1 pressure
  double frac_refine = 0.1, frac_coarsen = 0.05;
  int min_level = 0;
  int frac_type = 0;            // 0 fixed number, 1 fixed fraction (of the summed indicators)
  int64_t max_cells = 100000000;  // max number elements
  int max_level = 10;
};

Method parse_method(const std::string &s) {
  const char *names[] = {"steady", "bdf1", "bdf2", "bdf3", "sdirk2", "sdirk3"};
  for (int i = 0; i < 6; ++i)
    if (s == names[i]) return (Method)i;
  die("unknown time stepping method '%s'", s.c_str());
}

Params read_params(const Prm &p, int dim) {
  Params P;
  P.dim = dim;
  const std::string sc = "simulation control/";
  P.method = parse_method(p.get(sc + "method", "steady"));
  P.dt = p.d(sc + "time step", 1.0);
  P.t_end = p.d(sc + "time end", 1.0);
  P.startup = p.d(sc + "startup time scaling", 0.4);
  P.mesh_adapt = p.i(sc + "number mesh adapt", 0);
  P.output_frequency = p.i(sc + "output frequency", 1);
  P.log_frequency = p.i(sc + "log frequency", 1);
  P.subdivision = p.i(sc + "subdivision", 1);
  P.output_path = p.get(sc + "output path", "./");
  P.output_name = p.get(sc + "output name", "out");
  if (p.b(sc + "adapt", false)) die("adaptive time stepping is not supported");
  P.nu = p.d("physical properties/kinematic viscosity", 1.0);
  P.k = p.i("FEM/velocity order", 1);
  P.kp = p.i("FEM/pressure order", 1);
  P.qmapping_all = p.b("FEM/qmapping all", false);
  P.mesh_type = p.get("mesh/type", "dealii");
  if (P.mesh_type != "dealii" && P.mesh_type != "gmsh") die("mesh type '%s' is not supported (dealii | gmsh)", P.mesh_type.c_str());
  const std::string gt = p.get("mesh/grid type", "hyper_cube");
  P.grid_type = gt;
  P.grid_args = p.get("mesh/grid arguments", "-1 : 1 : false");
  P.mesh_file = p.get("mesh/file name", "none");
  P.general = P.mesh_type == "gmsh" || gt != "hyper_cube";
  {  // manifolds (source/core/manifolds.cc:133-186): spherical on boundary ids
    const int nm = p.i("manifolds/number", 0);
    for (int i = 0; i < nm; ++i) {
      const std::string ms = "manifolds/manifold " + std::to_string(i) + "/";
      Params::ManifoldPrm mp;
      mp.type = p.get(ms + "type", "none");
      mp.id = p.i(ms + "id", i);
      for (int a = 0; a < 3; ++a) mp.arg[a] = p.d(ms + "arg" + std::to_string(a + 1), 0.0);
      if (mp.type != "none" && mp.type != "spherical") die("manifold %d: type '%s' is not supported (none | spherical)", i, mp.type.c_str());
      P.manifolds.push_back(mp);
    }
  }
  P.display_precision = p.i("simulation control/display precision", 4);
  P.residual_precision = p.i("non-linear solver/residual precision", 4);
  if (!P.general) {
    const std::string a = P.grid_args;
    std::vector<std::string> parts;
    std::stringstream ss(a);
    std::string tok;
    while (std::getline(ss, tok, ':')) parts.push_back(trim(tok));
    if (parts.size() != 3) die("grid arguments '%s': expected 'lo : hi : colorize'", a.c_str());
    P.lo = std::atof(parts[0].c_str());
    P.hi = std::atof(parts[1].c_str());
    P.colorize = parts[2] == "true";
  }
  P.refinement = p.i("mesh/initial refinement", 0);
  const std::string madapt = p.get("mesh adaptation/type", "none");
  P.madapt = madapt;
  P.adapt_frequency = p.i("mesh adaptation/frequency", 1);
  if (P.adapt_frequency < 1) die("mesh adaptation/frequency must be >= 1");
  if (P.method == Method::steady && P.mesh_adapt > 0 && madapt != "uniform" && madapt != "kelly")
    die("mesh adaptation type '%s' is not supported (uniform or kelly)", madapt.c_str());
  if (madapt == "kelly") {  // refine_mesh_kelly (navier_stokes_base.cc:610-780)
    const std::string ma = "mesh adaptation/";
    const std::string var = p.get(ma + "variable", "velocity");
    if (var != "velocity" && var != "pressure") die("mesh adaptation variable '%s' is unknown", var.c_str());
    P.kelly_variable = var == "pressure" ? 1 : 0;
    const std::string ftype = p.get(ma + "fraction type", "number");
    if (ftype != "number" && ftype != "fraction") die("mesh adaptation: fraction type '%s' is unknown", ftype.c_str());
    P.frac_type = ftype == "fraction" ? 1 : 0;
    P.max_cells = (int64_t)p.d(ma + "max number elements", 100000000);
    P.frac_refine = p.d(ma + "fraction refinement", 0.1);
    P.max_level = p.i(ma + "max refinement level", 10);
    P.frac_coarsen = p.d(ma + "fraction coarsening", 0.05);
    P.min_level = p.i(ma + "min refinement level", 0);
    if (P.frac_refine < 0 || P.frac_coarsen < 0 || P.frac_refine + P.frac_coarsen > 1)
      die("mesh adaptation: fractions must be >= 0 with refinement + coarsening <= 1");
    if (P.k > 2 || P.kp > P.k) die("kelly mesh adaptation: 1 <= pressure order <= velocity order <= 2");
  }
  const int nbc = p.i("boundary conditions/number", 0);
  for (int i = 0; i < nbc; ++i) {
    const std::string s = "boundary conditions/bc " + std::to_string(i) + "/";
    BC b;
    b.type = p.get(s + "type", "noslip");
    b.id = p.i(s + "id", i);
    b.periodic_direction = p.i(s + "periodic_direction", 0);
    b.periodic_id = p.i(s + "periodic_id", 1);
    if (b.type == "function") {
      const char *nm[3] = {"u", "v", "w"};
      for (int c = 0; c < dim; ++c) b.f[c] = Function(p, s + nm[c], dim, "0");
    } else if (b.type != "noslip" && b.type != "periodic" && b.type != "slip") {
      die("bc %d: unknown type '%s'", i, b.type.c_str());
    }
    P.bcs.push_back(std::move(b));
  }
  const std::string zeros = dim == 3 ? "0; 0; 0; 0" : "0; 0; 0";
  P.source = p.b("source term/enable", false);
  if (P.source) P.force = Function(p, "source term/xyz", dim, zeros);
  P.ic_type = p.get("initial conditions/type", "nodal");
  P.ic = Function(p, "initial conditions/uvwp", dim, zeros);
  P.ic_nu = p.d("initial conditions/viscosity", 1.0);
  P.analytical = p.b("analytical solution/enable", false);
  P.analytical_verbose = p.get("analytical solution/verbosity", "quiet") == "verbose";
  P.analytical_file = p.get("analytical solution/filename", "L2Error");
  if (P.analytical) {  // the reference's subsection is "uvw" (analytical_solutions.cc:69-70); "uvwp" accepted too
    const bool uvw = p.get("analytical solution/uvw/Function expression", "\x01") != "\x01" ||
                     p.get("analytical solution/uvwp/Function expression", "\x01") == "\x01";
    P.exact = Function(p, uvw ? "analytical solution/uvw" : "analytical solution/uvwp", dim, zeros);
  }
  P.enstrophy = p.b("post-processing/calculate enstrophy", false);
  P.kinetic = p.b("post-processing/calculate kinetic energy", false);
  P.pp_verbose = p.get("post-processing/verbosity", "quiet") == "verbose";
  P.newton_tol = p.d("non-linear solver/tolerance", 1e-6);
  P.newton_max = p.i("non-linear solver/max iterations", 10);
  P.newton_verbose = p.get("non-linear solver/verbosity", "verbose") == "verbose" ? 1 : 0;
  {
    const std::string sv = p.get("non-linear solver/solver", "newton");
    if (sv == "skip_newton") P.nl_solver = GLS_SKIP_NEWTON;
    else if (sv != "newton") die("non-linear solver '%s' is unknown (newton|skip_newton)", sv.c_str());
    P.skip_iterations = p.i("non-linear solver/skip iterations", 1);
    if (P.skip_iterations < 1) die("non-linear solver/skip iterations must be >= 1");
  }
  P.lin_max = p.i("linear solver/max iters", 1000);
  P.lin_rel = p.d("linear solver/relative residual", 1e-3);
  P.lin_min = p.d("linear solver/minimum residual", 1e-8);
  // ILU(k) of the reference's GMRES (parameters.cc:546-560; a Double entry cast to Ifpack's integer
  // level of fill): integral values 0..GLS_ILU_MAX_FILL, anything else fails here
  {
    const double f = p.d("linear solver/ilu preconditioner fill", 0.0);
    if (!(f >= 0 && f <= GLS_ILU_MAX_FILL) || f != std::floor(f))
      die("linear solver/ilu preconditioner fill = %g is not supported (integers 0..%d)", f, GLS_ILU_MAX_FILL);
    P.ilu_fill = (int)f;
  }
  P.ilu_atol = p.d("linear solver/ilu preconditioner absolute tolerance", 1e-8);
  P.ilu_rtol = p.d("linear solver/ilu preconditioner relative tolerance", 1.0);
  // linear solver/method (parameters.cc:519-532, 616-626; dispatch gls_navier_stokes.cc:1140-1157):
  // gmres and bicgstab with the ILU(fill) of the entries above (or the geometric multigrid V-cycle where
  // the nested hyper_cube hierarchy exists); amg = GMRES + ML AMG with ILU smoother / coarsener
  // (setup_AMG, :1180-1240), which this library substitutes explicitly (announced at setup, see
  // Solver::announce_linear_solver): the geometric multigrid V-cycle on nested hyper_cubes, elsewhere
  // the ILU(amg preconditioner ilu fill / absolute / relative tolerance) that ML would smooth with.
  // The amg entries are validated (parameters.cc:562-595, 627-644) even where they do not act.
  {
    const std::string m = p.get("linear solver/method", "gmres");
    if (m == "gmres") P.lin_method = 0;
    else if (m == "bicgstab") P.lin_method = 1;
    else if (m == "amg") P.lin_method = 2;
    else die("linear solver/method '%s' is invalid (amg | gmres | bicgstab)", m.c_str());
    const double af = p.d("linear solver/amg preconditioner ilu fill", 0.0);
    if (!(af >= 0 && af <= GLS_ILU_MAX_FILL) || af != std::floor(af))
      die("linear solver/amg preconditioner ilu fill = %g is not supported (integers 0..%d)", af, GLS_ILU_MAX_FILL);
    P.amg_ilu_fill = (int)af;
    P.amg_ilu_atol = p.d("linear solver/amg preconditioner ilu absolute tolerance", 1e-12);
    P.amg_ilu_rtol = p.d("linear solver/amg preconditioner ilu relative tolerance", 1.0);
    P.amg_threshold = p.d("linear solver/amg aggregation threshold", 1e-14);
    P.amg_n_cycles = p.i("linear solver/amg n cycles", 1);
    P.amg_w_cycles = p.b("linear solver/amg w cycles", false);
    P.amg_sweeps = p.i("linear solver/amg smoother sweeps", 2);
    P.amg_overlap = p.i("linear solver/amg smoother overlap", 1);
    if (P.amg_n_cycles < 1) die("linear solver/amg n cycles must be >= 1");
    if (P.amg_sweeps < 0 || P.amg_overlap < 0) die("linear solver/amg smoother sweeps / overlap must be >= 0");
    if (P.amg_threshold < 0) die("linear solver/amg aggregation threshold must be >= 0");
    const std::string v = p.get("linear solver/verbosity", "verbose");
    if (v != "verbose" && v != "quiet") die("Unknown verbosity mode for the linear solver");
  }
  // restart (parameters.cc:759-798): checkpoint / restart files are out of scope; a prm
  // that asks for either fails here instead of silently running without it
  if (p.b("restart/restart", false)) die("restart/restart = true: restarting from a checkpoint is not supported");
  if (p.b("restart/checkpoint", false)) die("restart/checkpoint = true: checkpointing is not supported");
  P.timer = p.get("timer/type", "none");
  if (P.timer != "none" && P.timer != "iteration" && P.timer != "end") die("timer/type '%s' is unknown", P.timer.c_str());
  P.srf = p.get("velocity source/type", "none") == "srf";
  P.omega[0] = p.d("velocity source/omega_x", 0.);
  P.omega[1] = p.d("velocity source/omega_y", 0.);
  P.omega[2] = p.d("velocity source/omega_z", 0.);
  return P;
}

// ---------------------------------------------------------------------------------------------
// device CFL on box cells (calculate_CFL: |u| at the cell centre * dt / h_cell, h_cell =
// (6|K|/pi)^(1/3) / degree, 2D sqrt(4|K|/pi) / degree): one thread per cell, per-block maxima
// ---------------------------------------------------------------------------------------------
__global__ void k_cfl(const int32_t *cv, const double *h, const double *u, int64_t nc, int dim, int nvl, int k1,
                      double b0, double b1, double b2, double deg, double dt, double *blockmax) {
  __shared__ double red[256];
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double v = 0.0;
  if (c < nc) {
    const double B[3] = {b0, b1, b2};
    double uc[3] = {0, 0, 0}, meas = 1.0;
    for (int a = 0; a < nvl; ++a) {
      const int ax = a % k1, ay = (a / k1) % k1, az = a / (k1 * k1);
      const double w = B[ax] * B[ay] * (dim == 3 ? B[az] : 1.0);
      const int64_t node = cv[c * nvl + a];
      for (int d = 0; d < dim; ++d) uc[d] += w * u[node * dim + d];
    }
    for (int d = 0; d < dim; ++d) meas *= h[c * dim + d];
    const double hh = dim == 2 ? sqrt(4. * meas / M_PI) / deg : cbrt(6. * meas / M_PI) / deg;
    double un = 0;
    for (int d = 0; d < dim; ++d) un += uc[d] * uc[d];
    v = sqrt(un) / hh * dt;
  }
  red[threadIdx.x] = v;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + st]);
    __syncthreads();
  }
  if (threadIdx.x == 0) blockmax[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------------------------------------
// mesh and constraints
// ---------------------------------------------------------------------------------------------
struct Mesh {
  int dim = 3, n = 1, k = 1, kp = 1, pmask = 0;
  double lo = 0, hi = 1, hc = 1;
  int64_t nc = 0, nv = 0, np = 0;
  int vsh[3] = {1, 1, 1}, psh[3] = {1, 1, 1};  // lattice nodes per direction (periodic: wrapped)
  std::vector<int32_t> cv, cp;
  std::vector<double> x0, h;
  // locally refined mesh (gls_mesh_refined_create): explicit support points, hanging nodes and
  // their DoF-level constraint lines (empty on the uniform lattice)
  std::vector<double> vx, px;
  std::map<int, std::vector<double>> slip_normals;  // general meshes: boundary id -> node normals [nv][dim]
  std::map<int, std::vector<int32_t>> slip_rank;    // ... -> independent normal directions per node (edges, corners)
  std::map<int, std::vector<double>> slip_sets;     // ... -> the grouped normals [nv][3][dim]
  std::vector<uint8_t> vhanging;  // per velocity node
  std::vector<int64_t> hang_dofs, hang_off{0}, hang_master;
  std::vector<double> hang_w;
  // general (curved / unstructured) cells: MappingQ(k) support points per cell, cell->measure(),
  // boundary-id bits per velocity node (gls_umesh_fe_space)
  bool general = false;
  std::vector<double> support, measure;
  std::vector<uint32_t> vbid;
  int64_t n_dofs() const { return (int64_t)dim * nv + np; }
  // the DoFHandler's count deal.II prints on periodic meshes: periodicity is a constraint there, so the
  // nodes this build identifies are counted on both faces (-1: not periodic, n_dofs())
  int64_t n_dofs_dealii = -1;
  void coord(int64_t node, bool vel, double *x, int *idx) const {
    if (!vx.empty()) {  // refined mesh: no lattice index
      const double *src = &(vel ? vx : px)[(size_t)(node * dim)];
      for (int d = 0; d < dim; ++d) {
        x[d] = src[d];
        idx[d] = -1;
      }
      return;
    }
    const int *sh = vel ? vsh : psh;
    const int deg = vel ? k : kp;
    for (int d = 0; d < dim; ++d) {
      idx[d] = (int)(node % sh[d]);
      node /= sh[d];
      x[d] = lo + idx[d] * hc / deg;
    }
  }
};

Mesh build_mesh(const Params &P, int n, int pmask) {
  Mesh m;
  m.dim = P.dim;
  m.n = n;
  m.k = P.k;
  m.kp = P.kp;
  m.pmask = pmask;
  m.lo = P.lo;
  m.hi = P.hi;
  m.hc = (P.hi - P.lo) / n;
  ck(gls_mesh_hyper_cube_sizes(P.dim, n, P.k, P.kp, pmask, &m.nc, &m.nv, &m.np), "gls_mesh_hyper_cube_sizes");
  int nvl = 1, npl = 1;
  for (int d = 0; d < P.dim; ++d) {
    nvl *= P.k + 1;
    npl *= P.kp + 1;
  }
  for (int d = 0; d < 3; ++d) {
    const bool per = (pmask >> d) & 1;
    m.vsh[d] = P.k * n + (per ? 0 : 1);
    m.psh[d] = P.kp * n + (per ? 0 : 1);
  }
  m.cv.resize((size_t)(m.nc * nvl));
  m.cp.resize((size_t)(m.nc * npl));
  m.x0.resize((size_t)(m.nc * P.dim));
  m.h.resize((size_t)(m.nc * P.dim));
  ck(gls_mesh_hyper_cube(P.dim, n, P.k, P.kp, P.lo, P.hi, pmask, m.cv.data(), m.cp.data(), m.x0.data(), m.h.data()),
     "gls_mesh_hyper_cube");
  if (pmask) {  // deal.II's count: the unwrapped lattices
    int64_t nvf = 1, npf = 1;
    for (int d = 0; d < P.dim; ++d) {
      nvf *= (int64_t)P.k * n + 1;
      npf *= (int64_t)P.kp * n + 1;
    }
    m.n_dofs_dealii = (int64_t)P.dim * nvf + npf;
  }
  return m;
}

// the support point x lies on the box face lo (side 0) / hi (side 1) of axis d
bool on_face(const Mesh &m, const double *x, int d, int side) {
  const double tol = 1e-12 * (m.hi - m.lo);
  return std::fabs(x[d] - (side ? m.hi : m.lo)) <= tol;
}
// boundary ids of a support point (hyper_cube: colorize -> faces 2d / 2d+1, else all id 0)
unsigned face_bits(const Mesh &m, const double *x, bool colorize) {
  unsigned b = 0;
  for (int d = 0; d < m.dim; ++d) {
    if ((m.pmask >> d) & 1) continue;
    if (on_face(m, x, d, 0)) b |= 1u << (colorize ? 2 * d : 0);
    if (on_face(m, x, d, 1)) b |= 1u << (colorize ? 2 * d + 1 : 0);
  }
  return b;
}

struct Constraints {
  std::vector<uint8_t> mask;  // per velocity node, bit c = component c constrained
  std::vector<int64_t> dofs;
  std::vector<double> vals;
  // slip on curved walls (general meshes): n.u = 0 as the homogeneous line
  // u_c = -sum_{d != c} (n_d / n_c) u_d on the component c of largest |n_c| (DoF-level, like hanging lines)
  std::vector<int64_t> line_dofs, line_off{0}, line_master;
  std::vector<double> line_w;
};

// normal axes of the faces with boundary id `id` that node idx lies on (bit d = face normal e_d)
unsigned face_normals(const Mesh &m, const double *x, bool colorize, int id) {
  unsigned a = 0;
  for (int d = 0; d < m.dim; ++d) {
    if ((m.pmask >> d) & 1) continue;
    if (on_face(m, x, d, 0) && (colorize ? 2 * d : 0) == id) a |= 1u << d;
    if (on_face(m, x, d, 1) && (colorize ? 2 * d + 1 : 0) == id) a |= 1u << d;
  }
  return a;
}

// Dirichlet data of the noslip / function / slip boundary conditions at the velocity support
// points; a DoF already constrained by an earlier bc keeps its constraint (deal.II's first-constraint
// rule, per DoF: a slip line takes u_cmax only, later bcs still set the node's other components).
// slip = VectorTools::compute_no_normal_flux_constraints (gls_navier_stokes.cc:100-110, 149-160): on
// axis-aligned faces n.u = 0 constrains the normal component(s) to 0 (every face normal of this
// boundary at edges / corners); on curved walls it is the line u_cmax = -sum (n_d / n_cmax) u_d,
// added unless u_cmax is already constrained (masters that end up Dirichlet drop out of the closed
// operator lines, gls_set_hanging; a line whose master is itself a slip line is skipped, which
// keeps the lines free of cycles).
Constraints make_constraints(const Params &P, const Mesh &m, double t) {
  Constraints C;
  C.mask.assign((size_t)m.nv, 0);
  std::vector<uint8_t> lined((size_t)(m.nv * m.dim), 0);  // DoFs constrained by a slip line
  std::vector<double> val((size_t)(m.nv * m.dim), 0.0);
  for (const BC &b : P.bcs) {
    if (b.type == "periodic") continue;
    const std::vector<double> *sn = nullptr, *ss = nullptr;  // general meshes: node normals of this slip boundary
    const std::vector<int32_t> *sr = nullptr;
    if (b.type == "slip" && m.general) {
      auto it = m.slip_normals.find(b.id);
      if (it == m.slip_normals.end()) die("slip boundary %d: no node normals", b.id);
      sn = &it->second;
      sr = &m.slip_rank.at(b.id);
      ss = &m.slip_sets.at(b.id);
    }
    std::vector<int64_t> sel;
    std::vector<double> X;
    std::vector<unsigned> nrm;
    for (int64_t v = 0; v < m.nv; ++v) {
      double x[3];
      int idx[3];
      m.coord(v, true, x, idx);
      // hanging nodes keep their hanging constraint (interpolate_boundary_values skips DoFs that
      // are already constrained, gls_navier_stokes.cc:84-110)
      if (!m.vhanging.empty() && m.vhanging[(size_t)v]) continue;
      if ((m.general ? m.vbid[(size_t)v] : face_bits(m, x, P.colorize)) & (1u << b.id)) {
        sel.push_back(v);
        X.insert(X.end(), x, x + m.dim);
        const int rk = sr ? (*sr)[(size_t)v] : 0;
        if (sn && rk >= m.dim) {  // as many independent normals as components (a corner): u = 0
          nrm.push_back((1u << m.dim) - 1u);
        } else if (sn && rk == 2) {  // an edge in 3D: u parallel to t = n0 x n1, two constraints
          const double *g = &(*ss)[(size_t)(v * 3 * m.dim)];
          double t[3] = {0, 0, 0}, tl = 0;
          for (int j = 1; j < 3 && tl <= 1e-3; ++j) {
            const double *h = g + j * m.dim;
            t[0] = g[1] * h[2] - g[2] * h[1];
            t[1] = g[2] * h[0] - g[0] * h[2];
            t[2] = g[0] * h[1] - g[1] * h[0];
            tl = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
          }
          int cm = 0;
          for (int c = 1; c < 3; ++c)
            if (std::fabs(t[c]) > std::fabs(t[cm])) cm = c;
          unsigned ax = 0;
          for (int a = 0; a < 3; ++a) {
            if (a == cm) continue;
            const double w = t[a] / t[cm];
            if (std::fabs(w) < 1e-12) {  // t has no a-component: u_a = 0
              ax |= 1u << a;
              continue;
            }
            // u_a = (t_a / t_cm) u_cm, unless u_a is already constrained or u_cm carries a line
            if ((C.mask[(size_t)v] >> a) & 1u || lined[(size_t)(v * 3 + a)] || lined[(size_t)(v * 3 + cm)]) continue;
            C.line_dofs.push_back(v * 3 + a);
            C.line_master.push_back(v * 3 + cm);
            C.line_w.push_back(w);
            C.line_off.push_back((int64_t)C.line_master.size());
            lined[(size_t)(v * 3 + a)] = 1;
          }
          nrm.push_back(ax);
        } else if (sn) {  // n.u = 0: on a straight wall the normal is an axis and that component is 0
          unsigned ax = 0;
          bool axis = true;
          for (int c = 0; c < m.dim; ++c) {
            const double nc = std::fabs((*sn)[(size_t)(v * m.dim + c)]);
            if (nc > 1 - 1e-12) ax |= 1u << c;
            else if (nc > 1e-12) axis = false;
          }
          if (!axis) {  // curved wall: a constraint line on u_cmax (unless that DoF is already constrained)
            ax = 0;
            const double *n = &(*sn)[(size_t)(v * m.dim)];
            int cmax = 0;
            for (int c = 1; c < m.dim; ++c)
              if (std::fabs(n[c]) > std::fabs(n[cmax])) cmax = c;
            bool free_line = !((C.mask[(size_t)v] >> cmax) & 1u) && !lined[(size_t)(v * m.dim + cmax)];
            for (int d = 0; d < m.dim; ++d)
              if (d != cmax && std::fabs(n[d]) > 1e-14 && lined[(size_t)(v * m.dim + d)]) free_line = false;
            if (free_line) {
              C.line_dofs.push_back(v * m.dim + cmax);
              for (int d = 0; d < m.dim; ++d)
                if (d != cmax && std::fabs(n[d]) > 1e-14) {
                  C.line_master.push_back(v * m.dim + d);
                  C.line_w.push_back(-n[d] / n[cmax]);
                }
              C.line_off.push_back((int64_t)C.line_master.size());
              lined[(size_t)(v * m.dim + cmax)] = 1;
            }
          }
          nrm.push_back(ax);
        } else {
          nrm.push_back(face_normals(m, x, P.colorize, b.id));
        }
      }
    }
    std::vector<double> fv[3];
    if (b.type == "function")
      for (int c = 0; c < m.dim; ++c) b.f[c].eval(X, m.dim, t, fv[c]);
    for (size_t s = 0; s < sel.size(); ++s)
      for (int c = 0; c < m.dim; ++c) {
        uint8_t &mk = C.mask[(size_t)sel[s]];
        if (mk & (1u << c)) continue;
        if (lined[(size_t)(sel[s] * m.dim + c)]) continue;  // slip line first: the DoF keeps it
        if (b.type == "slip" && !((nrm[s] >> c) & 1u)) continue;
        mk |= (uint8_t)(1u << c);
        val[(size_t)(sel[s] * m.dim + c)] = b.type == "function" ? fv[c][s * (size_t)b.f[c].nc] : 0.0;
      }
  }
  for (int64_t v = 0; v < m.nv; ++v)
    for (int c = 0; c < m.dim; ++c)
      if (C.mask[(size_t)v] & (1u << c)) {
        C.dofs.push_back(v * m.dim + c);
        C.vals.push_back(val[(size_t)(v * m.dim + c)]);
      }
  return C;
}

// AffineConstraints::close() for the homogeneous lines: a master that is itself a constrained line
// (a hanging node's master vertex on a curved slip wall, whose u_cmax carries the slip line) is
// replaced by that line's masters with the weights multiplied; repeated masters are merged. Lines
// are acyclic (make_constraints), so the substitution ends after at most #lines rounds.
void close_lines(std::vector<int64_t> &ld, std::vector<int64_t> &lo, std::vector<int64_t> &lm,
                 std::vector<double> &lw) {
  std::unordered_map<int64_t, size_t> line_of;
  for (size_t i = 0; i < ld.size(); ++i) line_of[ld[i]] = i;
  bool chained = false;
  for (int64_t mj : lm) chained = chained || line_of.count(mj);
  if (!chained) return;
  std::vector<int64_t> no{0}, nm;
  std::vector<double> nw;
  for (size_t i = 0; i < ld.size(); ++i) {
    std::vector<std::pair<int64_t, double>> row, next;
    for (int64_t j = lo[i]; j < lo[i + 1]; ++j) row.emplace_back(lm[(size_t)j], lw[(size_t)j]);
    for (size_t round = 0;; ++round) {
      if (round > ld.size()) die("constraint lines: a cycle through DoF %lld", (long long)ld[i]);
      bool again = false;
      next.clear();
      for (auto [mj, w] : row) {
        auto it = line_of.find(mj);
        if (it == line_of.end()) { next.emplace_back(mj, w); continue; }
        again = true;
        const size_t l = it->second;
        for (int64_t j = lo[l]; j < lo[l + 1]; ++j) next.emplace_back(lm[(size_t)j], w * lw[(size_t)j]);
      }
      row.swap(next);
      if (!again) break;
    }
    std::map<int64_t, double> merged;
    for (auto [mj, w] : row) merged[mj] += w;
    for (auto [mj, w] : merged) {
      nm.push_back(mj);
      nw.push_back(w);
    }
    no.push_back((int64_t)nm.size());
  }
  lo.swap(no);
  lm.swap(nm);
  lw.swap(nw);
}

// ---------------------------------------------------------------------------------------------
// host quadrature for post-processing: Gauss points on [0,1], Lagrange on Gauss-Lobatto nodes
// ---------------------------------------------------------------------------------------------
void gauss01(int n, std::vector<double> &x, std::vector<double> &w) {
  x.assign((size_t)n, 0.);
  w.assign((size_t)n, 0.);
  for (int i = 0; i < n; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (n + 0.5)), dp = 1;
    for (int it = 0; it < 100; ++it) {
      double p0 = 1, p1 = 0;
      for (int j = 1; j <= n; ++j) {
        const double p2 = p1;
        p1 = p0;
        p0 = ((2 * j - 1) * z * p1 - (j - 1) * p2) / j;
      }
      dp = n * (z * p0 - p1) / (z * z - 1);
      const double dz = p0 / dp;
      z -= dz;
      if (std::fabs(dz) < 1e-16) break;
    }
    x[(size_t)(n - 1 - i)] = 0.5 * (z + 1);
    w[(size_t)(n - 1 - i)] = 1.0 / ((1 - z * z) * dp * dp);
  }
}
std::vector<double> lobatto01(int k) {
  if (k == 1) return {0., 1.};
  if (k == 2) return {0., .5, 1.};
  const double a = 0.5 * (1.0 - 1.0 / std::sqrt(5.0));
  return {0., a, 1. - a, 1.};
}
void lag1d(const std::vector<double> &xn, double x, double *v, double *dv) {
  const int n = (int)xn.size();
  for (int a = 0; a < n; ++a) {
    double val = 1, der = 0;
    for (int b = 0; b < n; ++b) {
      if (b == a) continue;
      const double f = (x - xn[(size_t)b]) / (xn[(size_t)a] - xn[(size_t)b]);
      der = der * f + val / (xn[(size_t)a] - xn[(size_t)b]);
      val *= f;
    }
    v[a] = val;
    dv[a] = der;
  }
}

// FE solution (velocity, gradient, pressure) at the tensor-product Gauss points of every cell
struct CellEval {
  const Mesh &m;
  int nq1, nq, nvl, npl;
  std::vector<double> xq, wq, Vv, Dv, Vp;  // 1D tables [q][node]
  CellEval(const Mesh &m_, int nq1d) : m(m_), nq1(nq1d) {
    gauss01(nq1, xq, wq);
    const std::vector<double> xv = lobatto01(m.k), xp = lobatto01(m.kp);
    const int k1 = m.k + 1, kp1 = m.kp + 1;
    Vv.resize((size_t)(nq1 * k1));
    Dv.resize((size_t)(nq1 * k1));
    Vp.resize((size_t)(nq1 * kp1));
    std::vector<double> tmp((size_t)kp1);
    for (int q = 0; q < nq1; ++q) {
      lag1d(xv, xq[(size_t)q], &Vv[(size_t)(q * k1)], &Dv[(size_t)(q * k1)]);
      lag1d(xp, xq[(size_t)q], &Vp[(size_t)(q * kp1)], tmp.data());
    }
    nq = m.dim == 3 ? nq1 * nq1 * nq1 : nq1 * nq1;
    nvl = m.dim == 3 ? k1 * k1 * k1 : k1 * k1;
    npl = m.dim == 3 ? kp1 * kp1 * kp1 : kp1 * kp1;
  }
  void qidx(int q, int *qq) const {
    qq[0] = q % nq1;
    qq[1] = (q / nq1) % nq1;
    qq[2] = m.dim == 3 ? q / (nq1 * nq1) : 0;
  }
  // MappingQ(k) of a general cell at Gauss point q: x, J^-1 [a][i], det J (k <= 2: equidistant)
  void mapped(int64_t c, int q, double *x, double JI[3][3], double &det) const {
    const int dim = m.dim, k1 = m.k + 1;
    int qq[3];
    qidx(q, qq);
    double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int d = 0; d < 3; ++d) x[d] = 0;
    const double *S = &m.support[(size_t)(c * nvl * dim)];
    for (int b = 0; b < nvl; ++b) {
      const int b0 = b % k1, b1 = (b / k1) % k1, b2 = dim == 3 ? b / (k1 * k1) : 0;
      const double v0 = Vv[(size_t)(qq[0] * k1 + b0)], v1 = Vv[(size_t)(qq[1] * k1 + b1)];
      const double v2 = dim == 3 ? Vv[(size_t)(qq[2] * k1 + b2)] : 1.0;
      const double g[3] = {Dv[(size_t)(qq[0] * k1 + b0)] * v1 * v2, v0 * Dv[(size_t)(qq[1] * k1 + b1)] * v2,
                           dim == 3 ? v0 * v1 * Dv[(size_t)(qq[2] * k1 + b2)] : 0.0};
      for (int i = 0; i < dim; ++i) {
        x[i] += S[b * dim + i] * v0 * v1 * v2;
        for (int a = 0; a < dim; ++a) J[i][a] += S[b * dim + i] * g[a];
      }
    }
    if (dim == 2) {
      det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
      JI[0][0] = J[1][1] / det; JI[0][1] = -J[0][1] / det; JI[1][0] = -J[1][0] / det; JI[1][1] = J[0][0] / det;
    } else {
      det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) - J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
            J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
      for (int a = 0; a < 3; ++a)
        for (int i = 0; i < 3; ++i)
          JI[a][i] = (J[(i + 1) % 3][(a + 1) % 3] * J[(i + 2) % 3][(a + 2) % 3] -
                      J[(i + 1) % 3][(a + 2) % 3] * J[(i + 2) % 3][(a + 1) % 3]) / det;
    }
  }
  void point(int64_t c, int q, double *x, double &JxW) const {
    int qq[3];
    qidx(q, qq);
    if (m.general) {
      double JI[3][3], det;
      mapped(c, q, x, JI, det);
      JxW = det * wq[(size_t)qq[0]] * wq[(size_t)qq[1]] * (m.dim == 3 ? wq[(size_t)qq[2]] : 1.0);
      return;
    }
    JxW = 1;
    for (int d = 0; d < m.dim; ++d) {
      const double hd = m.h[(size_t)(c * m.dim + d)];
      x[d] = m.x0[(size_t)(c * m.dim + d)] + hd * xq[(size_t)qq[d]];
      JxW *= hd * wq[(size_t)qq[d]];
    }
  }
  double phi_v(int a, const int *qq) const {
    const int k1 = m.k + 1, a0 = a % k1, a1 = (a / k1) % k1, a2 = m.dim == 3 ? a / (k1 * k1) : 0;
    return Vv[(size_t)(qq[0] * k1 + a0)] * Vv[(size_t)(qq[1] * k1 + a1)] * (m.dim == 3 ? Vv[(size_t)(qq[2] * k1 + a2)] : 1.);
  }
  double phi_p(int a, const int *qq) const {
    const int k1 = m.kp + 1, a0 = a % k1, a1 = (a / k1) % k1, a2 = m.dim == 3 ? a / (k1 * k1) : 0;
    return Vp[(size_t)(qq[0] * k1 + a0)] * Vp[(size_t)(qq[1] * k1 + a1)] * (m.dim == 3 ? Vp[(size_t)(qq[2] * k1 + a2)] : 1.);
  }
  void at(const double *sol, int64_t c, int q, double *u, double G[3][3], double &p) const {
    const int dim = m.dim, k1 = m.k + 1;
    int qq[3];
    qidx(q, qq);
    const double one[3] = {1.0, 1.0, 1.0};
    const double *hh = m.general ? one : &m.h[(size_t)(c * dim)];
    double JI[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    if (m.general) {
      double x[3], det;
      mapped(c, q, x, JI, det);
    }
    for (int d = 0; d < 3; ++d) {
      u[d] = 0;
      for (int e = 0; e < 3; ++e) G[d][e] = 0;
    }
    p = 0;
    const int32_t *cv = &m.cv[(size_t)(c * nvl)];
    for (int a = 0; a < nvl; ++a) {
      const int a0 = a % k1, a1 = (a / k1) % k1, a2 = dim == 3 ? a / (k1 * k1) : 0;
      const double b0 = Vv[(size_t)(qq[0] * k1 + a0)], b1 = Vv[(size_t)(qq[1] * k1 + a1)];
      const double b2 = dim == 3 ? Vv[(size_t)(qq[2] * k1 + a2)] : 1.0;
      const double gr[3] = {Dv[(size_t)(qq[0] * k1 + a0)] * b1 * b2 / hh[0], b0 * Dv[(size_t)(qq[1] * k1 + a1)] * b2 / hh[1],
                            dim == 3 ? b0 * b1 * Dv[(size_t)(qq[2] * k1 + a2)] / hh[2] : 0.0};
      double g[3] = {gr[0], gr[1], gr[2]};
      if (m.general)
        for (int i = 0; i < dim; ++i) {
          g[i] = 0.0;
          for (int e = 0; e < dim; ++e) g[i] += JI[e][i] * gr[e];
        }
      for (int d = 0; d < dim; ++d) {
        const double ud = sol[(size_t)cv[a] * dim + d];
        u[d] += ud * b0 * b1 * b2;
        for (int e = 0; e < dim; ++e) G[d][e] += ud * g[e];
      }
    }
    const int32_t *cp = &m.cp[(size_t)(c * npl)];
    const int64_t voff = (int64_t)dim * m.nv;
    for (int a = 0; a < npl; ++a) p += sol[(size_t)(voff + cp[a])] * phi_p(a, qq);
  }
};

// ---------------------------------------------------------------------------------------------
// the solver
// ---------------------------------------------------------------------------------------------

// ---------------------------------------------------------------------------------------------
// `--np N`: the reference's `mpirun -np N gls_navier_stokes_{2d,3d} file.prm`
// (applications/gls_navier_stokes_3d/gls_navier_stokes_3d.cc:32-33) without MPI: the program forks
// N processes before any GPU call, one rank each (GPU rank % devices). Every rank holds the same
// host-side triangulation, constraints and time loop (replicated, deterministic); the GPU work --
// assembly, Jacobian action, GMRES / Newton, the ILU of its owned rows -- runs on the rank's cells
// only (gls_gpart_* + gls_dist_attach_dofs, the p::d partition of navier_stokes_base.cc:55-60,
// re-done after every adaptation). Ghost exchange and dot-product reductions go over RCCL when
// every rank has its own GPU (gls_dist_attach_dofs_rccl), else through this host shared-memory
// transport (callbacks: device -> host slot, barrier, peers' slots -> device). Host-side gathers
// of the global solution (post-processing, Kelly, output) use the same shared memory.
// ---------------------------------------------------------------------------------------------
constexpr int kMaxRanks = 64;
struct ShmComm {
  struct Header {
    std::atomic<int> count, gen, abort;
    unsigned char rccl_id[GLS_RCCL_ID_BYTES];
    int64_t nbar[kMaxRanks];   // barriers entered per rank and the tag of the last one (watchdog report)
    char tag[kMaxRanks][24];
    int64_t table[kMaxRanks][kMaxRanks][2];  // exchange mailbox: (start, count) of rank s's data for rank d
  };
  static constexpr size_t kSlot = (size_t)1 << 26;  // doubles per rank slot (virtual, NORESERVE)
  static constexpr size_t kGlob = (size_t)1 << 27;  // doubles of the shared global vector
  Header *hdr = nullptr;
  double *slots = nullptr, *glob = nullptr;
  int rank = 0, world = 1;
  void create(int w) {
    world = w;
    const size_t bytes = sizeof(Header) + (size_t)w * kSlot * sizeof(double) + kGlob * sizeof(double) + 4096;
    void *mem = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (mem == MAP_FAILED) die("--np: shared memory of %zu bytes not available", bytes);
    hdr = new (mem) Header();
    hdr->count.store(0);
    hdr->gen.store(0);
    hdr->abort.store(0);
    g_abort = &hdr->abort;
    char *base = static_cast<char *>(mem) + ((sizeof(Header) + 4095) / 4096) * 4096;
    slots = reinterpret_cast<double *>(base);
    glob = slots + (size_t)w * kSlot;
  }
  double *slot(int r) const { return slots + (size_t)r * kSlot; }
  // sense-reversing; a rank that failed raises abort. Watchdog: when NO rank has entered a barrier for
  // GLS_NP_WATCHDOG seconds (default 600) while this one waits -- a stall, not merely long rank-local
  // work (output, Kelly, ILU setup on big meshes) -- it reports every rank's barrier count and last
  // tag (ranks that disagree name the collective one of them skipped) and aborts the run.
  void barrier(const char *tag = "") const {
    ++hdr->nbar[rank];
    std::snprintf(hdr->tag[rank], sizeof(hdr->tag[rank]), "%s", tag);
    const int g = hdr->gen.load();
    if (hdr->count.fetch_add(1) == world - 1) {
      hdr->count.store(0);
      hdr->gen.fetch_add(1);
      return;
    }
    static const double limit = std::getenv("GLS_NP_WATCHDOG") ? std::atof(std::getenv("GLS_NP_WATCHDOG")) : 600.0;
    auto progress = [&]() {
      int64_t t = 0;
      for (int r = 0; r < world; ++r) t += hdr->nbar[r];
      return t;
    };
    auto t0 = std::chrono::steady_clock::now();
    int64_t seen = progress();
    for (uint64_t spin = 0; hdr->gen.load() == g; ++spin) {
      if (hdr->abort.load()) _exit(3);
      sched_yield();
      if ((spin & 4095) == 0 && progress() != seen) {  // another rank reached a barrier: not stalled
        seen = progress();
        t0 = std::chrono::steady_clock::now();
      }
      if ((spin & 4095) == 0 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
        std::fprintf(stderr, "--np watchdog: rank %d waited %.0f s at barrier #%lld (%s); ranks:", rank, limit,
                     (long long)hdr->nbar[rank], tag);
        for (int r = 0; r < world; ++r) std::fprintf(stderr, " [%d] #%lld %s", r, (long long)hdr->nbar[r], hdr->tag[r]);
        std::fprintf(stderr, "\n");
        hdr->abort.store(1);
        _exit(3);
      }
    }
  }
  // every rank writes values[i] at global position idx[i]; all receive the whole vector
  void allgather(const double *values, const std::vector<int64_t> &idx, std::vector<double> &out) const {
    if ((size_t)out.size() > kGlob) die("--np: global vector of %zu values exceeds the shared area", out.size());
    for (size_t i = 0; i < idx.size(); ++i) glob[idx[i]] = values[i];
    barrier("allgather");
    std::memcpy(out.data(), glob, out.size() * sizeof(double));
    barrier("allgather-done");
  }
  void bcast(std::vector<double> &v, int root) const {  // v sized alike on every rank
    if (rank == root) std::memcpy(glob, v.data(), v.size() * sizeof(double));
    barrier("bcast");
    if (rank != root) std::memcpy(v.data(), glob, v.size() * sizeof(double));
    barrier("bcast-done");
  }
};
ShmComm g_comm;

// host-staged exchange of one distributed context (gls_dist_attach_dofs callbacks)
struct ShmExchange {
  std::vector<int> nbrs;
  std::vector<int64_t> soff, roff;
  double *send = nullptr, *recv = nullptr, *red = nullptr;  // device buffers
  std::vector<double> tmp;
  ~ShmExchange() {
    for (double *q : {send, recv, red})
      if (q) (void)hipFree(q);
  }
  static int exchange(void *user, int phase) {
    auto *x = static_cast<ShmExchange *>(user);
    const ShmComm &C = g_comm;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    const std::vector<int64_t> &so = phase == 0 ? x->soff : x->roff, &ro = phase == 0 ? x->roff : x->soff;
    double *src = phase == 0 ? x->send : x->recv, *dst = phase == 0 ? x->recv : x->send;
    const int64_t ns = so.back();
    if ((size_t)ns > ShmComm::kSlot) return -1;
    if (ns && hipMemcpy(C.slot(C.rank), src, sizeof(double) * (size_t)ns, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    for (size_t i = 0; i < x->nbrs.size(); ++i) {
      C.hdr->table[C.rank][x->nbrs[i]][0] = so[i];
      C.hdr->table[C.rank][x->nbrs[i]][1] = so[i + 1] - so[i];
    }
    C.barrier(phase == 0 ? "import" : "export-add");
    for (size_t i = 0; i < x->nbrs.size(); ++i) {
      const int s = x->nbrs[i];
      const int64_t start = C.hdr->table[s][C.rank][0], cnt = C.hdr->table[s][C.rank][1];
      if (cnt != ro[i + 1] - ro[i]) return -1;
      if (cnt && hipMemcpy(dst + ro[i], C.slot(s) + start, sizeof(double) * (size_t)cnt, hipMemcpyHostToDevice) != hipSuccess)
        return -1;
    }
    C.barrier(phase == 0 ? "import-done" : "export-add-done");
    return 0;
  }
  static int allreduce(void *user, double *dev, int n) {
    auto *x = static_cast<ShmExchange *>(user);
    const ShmComm &C = g_comm;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpy(C.slot(C.rank), dev, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    C.barrier("allreduce");
    x->tmp.assign((size_t)n, 0.0);
    for (int r = 0; r < C.world; ++r)  // rank order: the same sum on every rank
      for (int i = 0; i < n; ++i) x->tmp[(size_t)i] += C.slot(r)[i];
    C.barrier("allreduce-done");
    return hipMemcpy(dev, x->tmp.data(), sizeof(double) * (size_t)n, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
  }
};

// TimerOutput(pcout, summary, wall_times) of NavierStokesBase (navier_stokes_base.cc:63-66): named
// sections with call counts and wall seconds (device work drained at the section boundaries),
// printed as deal.II's TimerOutput::print_summary table; output disabled for timer/type = none
// (navier_stokes_base.cc:97-98), per iteration with a reset (:449-455), and at destruction.
struct SectionTimer {
  bool on = false;
  std::map<std::string, std::pair<int, double>> sec;  // name -> (calls, wall seconds), name order
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  struct Scope {
    SectionTimer &T;
    std::string name;
    std::chrono::steady_clock::time_point a;
    Scope(SectionTimer &t, const char *n) : T(t), name(n) {
      if (T.on) {
        (void)hipDeviceSynchronize();
        a = std::chrono::steady_clock::now();
      }
    }
    ~Scope() {
      if (!T.on) return;
      (void)hipDeviceSynchronize();
      T.add(name, 1, std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count());
    }
  };
  void add(const std::string &name, int calls, double seconds) {
    auto &e = sec[name];
    e.first += calls;
    e.second += seconds;
  }
  void reset() {
    sec.clear();
    t0 = std::chrono::steady_clock::now();
  }
  void print() const {
    if (!on) return;
    const double total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::ostringstream o;
    o << "\n\n+---------------------------------------------+------------+------------+\n"
      << "| Total wallclock time elapsed since start    |";
    o << std::setw(10) << std::setprecision(3) << std::right << total << "s |            |\n";
    o << "|                                             |            |            |\n";
    o << "| Section                         | no. calls |  wall time | % of total |\n";
    o << "+---------------------------------+-----------+------------+------------+";
    for (const auto &e : sec) {
      std::string name = e.first;
      name.resize(32, ' ');
      o << "\n| " << name << "| " << std::setw(9) << e.second.first << " |" << std::setw(10) << std::setprecision(3)
        << e.second.second << "s |" << std::setw(10);
      const double f = total > 0 ? e.second.second / total : 0.0;
      if (f > 0.001) o << std::setprecision(2) << f * 100;
      else o << 0.0;
      o << "% |";
    }
    o << "\n+---------------------------------+-----------+------------+------------+\n\n";
    std::fputs(o.str().c_str(), stdout);
  }
};

struct Solver {
  Params &P;
  bool use_mg;
  SectionTimer timer;
  // --np: this process's rank, the rank count, the RCCL communicator (one GPU per rank) and the
  // rank-local part of the current mesh (local DoF -> global DoF, owned DoFs, transport state)
  int rank = 0, world = 1;
  gls_rccl *rccl = nullptr;
  struct Local {
    std::vector<int64_t> l2g, g2l, own_l, own_g;
    std::unique_ptr<ShmExchange> xchg;
    std::vector<double> tmp;
  } loc;
  int64_t ndev() const { return world > 1 ? (int64_t)loc.l2g.size() : m.n_dofs(); }
  Mesh m;
  Constraints C;
  std::vector<std::vector<int64_t>> g_lines;  // the current mesh's global constraint lines (dofs, offsets, masters)
  std::vector<double> g_lines_w;
  gls_ctx *ctx = nullptr;
  gls_refined_mesh *rmesh = nullptr;  // the adapted mesh m was built from (kelly; gls_octree_mesh)
  gls_octree *tree = nullptr;         // kelly: the forest p4est keeps (created at the first adaptation)
  gls_umesh *um = nullptr;            // general meshes: the triangulation (kept across refinements)
  gls_fe_space *space = nullptr;      // and its current FE space
  std::vector<gls_ctx *> mg_levels;
  double *d_present = nullptr, *d_m1 = nullptr, *d_m2 = nullptr, *d_m3 = nullptr;
  std::vector<double> present, m1, m2, m3;
  // The time loop is device-resident: between solves the state and history live in d_* (history
  // shift = pointer rotation + one device copy, CFL on the device for box meshes); the host copies
  // are refreshed only for output, post-processing, mesh adaptation and initial conditions.
  bool dev_ok = false, host_ok = true;  // which side holds the current state
  int32_t *d_cv = nullptr;              // box meshes: cell -> velocity node map and extents (device CFL)
  double *d_h = nullptr, *d_blk = nullptr;
  int step = 0;
  double time = 0.0, dt_now = 0.0, cfl = 0.0;
  double dts[4] = {0, 0, 0, 0};  // time steps, most recent first (BDF coefficients)
  int newton_its = 0, linear_its = 0;
  std::vector<std::vector<double>> errors;  // steady: cells, e_u, e_p ; transient: t, e_u
  std::vector<std::pair<double, std::string>> pvd;

  int precision = 4;    // error-table digits (ConvergenceTable scientific precision)
  bool stats = false;   // print the solver iteration totals at the end (--stats)
  static std::string g6(double v) {  // std::ostream's default formatting (6 significant digits)
    char b[64];
    std::snprintf(b, sizeof(b), "%g", v);
    return b;
  }
  Solver(Params &p, bool mg) : P(p), use_mg(mg), use_ilu(mg) { timer.on = P.timer != "none"; }
  bool use_ilu;              // assembled ILU(0) where no multigrid hierarchy exists (--precond jacobi: off)
  int forest_mode = 0;       // adapted meshes: 0 default, 1 --precond ilu (never the hierarchy multigrid),
                             // 2 --precond hmg (the hierarchy multigrid for every method and order)
  gls_ctx *ilu_ctx = nullptr;  // the context the ILU was attached to (a new mesh builds a new context)
  int64_t ilu_block_dofs = 0;  // block-Jacobi ILU subdomain size (0: one block, the single-rank reference)
  std::string dump_dir;        // --dump DIR: the state of every iteration's last solve (test hook)
  int last_scheme = GLS_STEADY;
  double last_ts[4] = {1, 1, 1, 1};
  // --dump: after an iteration, the last nonlinear solve's scheme, time steps, mesh size and its
  // present solution + history (raw little-endian float64, n_dofs each) as DIR/iterNNNN.{meta,bin}
  void dump_state() {
    if (dump_dir.empty()) return;
    need_host();
    if (rank != 0) return;
    char b[64];
    std::snprintf(b, sizeof(b), "/iter%04d", step);
    const std::string stem = dump_dir + b;
    FILE *f = std::fopen((stem + ".meta").c_str(), "w");
    if (!f) die("--dump: cannot write %s.meta", stem.c_str());
    std::fprintf(f, "step %d\ntime %.17g\nscheme %d\nn_cells %lld\nn_dofs %lld\ntime_steps %.17g %.17g %.17g %.17g\n", step,
                 time, last_scheme, (long long)m.nc, (long long)m.n_dofs(), last_ts[0], last_ts[1], last_ts[2], last_ts[3]);
    std::fclose(f);
    f = std::fopen((stem + ".bin").c_str(), "wb");
    if (!f) die("--dump: cannot write %s.bin", stem.c_str());
    for (const std::vector<double> *v : {&present, &m1, &m2, &m3}) std::fwrite(v->data(), sizeof(double), v->size(), f);
    std::fclose(f);
  }
  int ilu_order = -1;  // --ilu-order cm|multicolor (-1: by size, kIluMulticolorDofs)
  static constexpr int64_t kIluMulticolorDofs = 100000;
  ~Solver() {
    release();
    if (space) gls_fe_space_destroy(space);
    if (um) gls_umesh_destroy(um);
    if (tree) gls_octree_destroy(tree);
  }

  void release() {
    for (gls_ctx *g : mg_levels) gls_destroy(g);
    mg_levels.clear();
    for (gls_refined_mesh *R : mg_meshes) gls_octree_mesh_destroy(R);
    mg_meshes.clear();
    if (ctx) gls_destroy(ctx);
    ilu_ctx = nullptr;
    ctx = nullptr;
    loc.xchg.reset();  // the transport outlives its context
    if (rmesh) gls_octree_mesh_destroy(rmesh);
    rmesh = nullptr;
    if (d_cv) (void)hipFree(d_cv);
    for (double *q : {d_h, d_blk}) if (q) (void)hipFree(q);
    d_cv = nullptr;
    d_h = d_blk = nullptr;
    for (double *q : {d_present, d_m1, d_m2, d_m3})
      if (q) (void)hipFree(q);
    d_present = d_m1 = d_m2 = d_m3 = nullptr;
  }

  int periodic_mask() const {
    int pm = 0;
    for (const BC &b : P.bcs)
      if (b.type == "periodic") pm |= 1 << b.periodic_direction;
    return pm;
  }

  gls_ctx *make_context(const Mesh &mm, const Constraints &cc) {
    std::vector<double> fq;
    if (P.source && !mm.general) {  // source term at the quadrature points QGauss(k+1)
      CellEval ev(mm, mm.k + 1);
      std::vector<double> X, F;
      X.reserve((size_t)(mm.nc * ev.nq * mm.dim));
      for (int64_t c = 0; c < mm.nc; ++c)
        for (int q = 0; q < ev.nq; ++q) {
          double x[3], w;
          ev.point(c, q, x, w);
          X.insert(X.end(), x, x + mm.dim);
        }
      P.force.eval(X, mm.dim, time, F);
      fq.resize(X.size());
      for (size_t i = 0; i < fq.size() / mm.dim; ++i)
        for (int d = 0; d < mm.dim; ++d) fq[i * mm.dim + d] = F[i * (size_t)P.force.nc + d];
    }
    gls_mesh_desc D;
    std::memset(&D, 0, sizeof(D));
    D.dim = mm.dim;
    D.k = mm.k;
    D.kp = mm.kp;
    D.n_cells = (int)mm.nc;
    D.n_vnodes = (int)mm.nv;
    D.n_pnodes = (int)mm.np;
    D.cell_vnodes = mm.cv.data();
    if (mm.kp == mm.k && (mm.cp != mm.cv || mm.np != mm.nv)) die("equal-order mesh with distinct pressure nodes");
    D.cell_pnodes = (mm.kp == mm.k) ? nullptr : mm.cp.data();
    if (mm.general) {  // MappingQ(k) support points (gls_umesh_fe_space)
      D.map_degree = mm.k;
      D.cell_support = mm.support.data();
    } else {
      D.cell_x0 = mm.x0.data();
      D.cell_h = mm.h.data();
    }
    D.vnode_mask = cc.mask.data();
    D.viscosity = P.nu;
    D.srf = P.srf ? 1 : 0;
    for (int i = 0; i < 3; ++i) D.omega[i] = P.omega[i];
    D.force_q = (P.source && !mm.general) ? fq.data() : nullptr;
    gls_ctx *g = nullptr;
    ck(gls_create(&D, &g), "gls_create");
    if (P.source && mm.general) {  // forcing at the library's (mapped) quadrature points
      const int nq1 = mm.k + 1, nq = mm.dim == 3 ? nq1 * nq1 * nq1 : nq1 * nq1;
      std::vector<double> X((size_t)(mm.nc * nq * mm.dim)), F;
      ck(gls_quadrature_points(g, X.data()), "gls_quadrature_points");
      P.force.eval(X, mm.dim, time, F);
      fq.resize(X.size());
      for (size_t i = 0; i < fq.size() / mm.dim; ++i)
        for (int d = 0; d < mm.dim; ++d) fq[i * mm.dim + d] = F[i * (size_t)P.force.nc + d];
      ck(gls_set_force(g, fq.data()), "gls_set_force");
    }
    ck(gls_set_dirichlet(g, (int64_t)cc.dofs.size(), cc.dofs.data(), cc.vals.data()), "gls_set_dirichlet");
    return g;
  }

  // --np: the rank's context on its cells of a general mesh (gls_gpart_*), Dirichlet rows mapped to
  // local DoFs, attached to RCCL or the shared-memory transport; lines (global DoF ids) decide the
  // ghosts (their masters) and are set by the caller through loc.g2l
  gls_ctx *make_context_local(const Mesh &mm, const Constraints &cc, const std::vector<int64_t> &ld,
                              const std::vector<int64_t> &lo, const std::vector<int64_t> &lm) {
    const bool sep = mm.kp != mm.k;
    const int dim = mm.dim, nvc = dim == 3 ? (mm.k + 1) * (mm.k + 1) * (mm.k + 1) : (mm.k + 1) * (mm.k + 1);
    const int npc = dim == 3 ? (mm.kp + 1) * (mm.kp + 1) * (mm.kp + 1) : (mm.kp + 1) * (mm.kp + 1);
    // what a p::d triangulation hands this rank (dist.py local_part, the gls_dpart_create contract): its owned
    // cells (the equal-count range of the cell order) plus the ghost layer -- every cell touching a node of an
    // owned cell, a master of a line on one, or the DoF node of a line one of whose masters it touches -- with
    // owners, node keys (= the global node ids) and those cells' lines in DoF keys; the partition is built
    // from that part alone (gls_dpart_create), not from the global arrays
    const int64_t cb = mm.nc * rank / world, ce = mm.nc * (rank + 1) / world, NVD0 = (int64_t)dim * mm.nv;
    const int64_t nun = mm.nv + (sep ? mm.np : 0);
    auto unode = [&](int64_t g) { return g < NVD0 ? g / dim : (sep ? mm.nv : 0) + g - NVD0; };  // DoF -> node
    auto dkey = [&](int64_t g) {  // DoF -> DoF key (node key * (dim + 1) + component, dim for pressure)
      return g < NVD0 ? (g / dim) * (dim + 1) + g % dim : (g - NVD0) * (dim + 1) + dim;
    };
    auto cell_touch = [&](int64_t c, const std::vector<uint8_t> &S) {
      for (int a = 0; a < nvc; ++a)
        if (S[(size_t)mm.cv[(size_t)(c * nvc + a)]]) return true;
      if (sep)
        for (int a = 0; a < npc; ++a)
          if (S[(size_t)(mm.nv + mm.cp[(size_t)(c * npc + a)])]) return true;
      return false;
    };
    std::vector<uint8_t> S((size_t)nun, 0);
    for (int64_t c = cb; c < ce; ++c) {
      for (int a = 0; a < nvc; ++a) S[(size_t)mm.cv[(size_t)(c * nvc + a)]] = 1;
      if (sep)
        for (int a = 0; a < npc; ++a) S[(size_t)(mm.nv + mm.cp[(size_t)(c * npc + a)])] = 1;
    }
    {
      std::vector<uint8_t> add(S);
      for (size_t i = 0; i < ld.size(); ++i)
        for (int64_t j = lo[i]; j < lo[i + 1]; ++j) {
          const int64_t dn = unode(ld[i]), mn = unode(lm[(size_t)j]);
          if (S[(size_t)dn]) add[(size_t)mn] = 1;  // masters of the lines on the owned cells' nodes
          if (S[(size_t)mn]) add[(size_t)dn] = 1;  // DoF nodes of the lines whose master an owned cell touches
        }
      S.swap(add);
    }
    std::vector<int32_t> powner;
    std::vector<int64_t> pvk, ppk;
    std::vector<uint8_t> pnode((size_t)nun, 0);
    for (int64_t c = 0; c < mm.nc; ++c) {
      if (!cell_touch(c, S)) continue;
      int r = (int)std::min<int64_t>(world - 1, c * world / std::max<int64_t>(mm.nc, 1));
      while (r > 0 && c < mm.nc * r / world) --r;
      while (r < world - 1 && c >= mm.nc * (r + 1) / world) ++r;
      powner.push_back(r);
      for (int a = 0; a < nvc; ++a) {
        pvk.push_back(mm.cv[(size_t)(c * nvc + a)]);
        pnode[(size_t)mm.cv[(size_t)(c * nvc + a)]] = 1;
      }
      if (sep)
        for (int a = 0; a < npc; ++a) {
          ppk.push_back(mm.cp[(size_t)(c * npc + a)]);
          pnode[(size_t)(mm.nv + mm.cp[(size_t)(c * npc + a)])] = 1;
        }
    }
    std::vector<int64_t> lkd, lko{0}, lkm;  // the part's lines (DoF node on a provided cell), in DoF keys
    for (size_t i = 0; i < ld.size(); ++i) {
      if (!pnode[(size_t)unode(ld[i])]) continue;
      lkd.push_back(dkey(ld[i]));
      for (int64_t j = lo[i]; j < lo[i + 1]; ++j) lkm.push_back(dkey(lm[(size_t)j]));
      lko.push_back((int64_t)lkm.size());
    }
    gls_gpart *gp = nullptr;
    ck(gls_dpart_create(dim, mm.k, mm.kp, (int64_t)powner.size(), powner.data(), pvk.data(), sep ? ppk.data() : nullptr,
                        (int64_t)lkd.size(), lkd.data(), lko.data(), lkm.data(), rank, world, &gp),
       "gls_dpart_create");
    int64_t cb_l, ce_l, nvl, npl, nov, nop, ns, nr;
    int nn;
    ck(gls_gpart_sizes(gp, &cb_l, &ce_l, &nvl, &npl, &nov, &nop, &nn, &ns, &nr), "gls_gpart_sizes");
    const int64_t ncl = ce_l - cb_l;
    if (ncl != ce - cb) die("--np: the local part's owned cells (%lld) differ from the rank's range (%lld)", (long long)ncl,
                            (long long)(ce - cb));
    std::vector<int32_t> lcv((size_t)(ncl * nvc)), lcp(sep ? (size_t)(ncl * npc) : 0), sd((size_t)ns), rd((size_t)nr);
    std::vector<int64_t> vl2g((size_t)nvl), pl2g((size_t)npl), soff((size_t)nn + 1, 0), roff((size_t)nn + 1, 0);
    std::vector<int> nbrs((size_t)nn);
    ck(gls_gpart_get(gp, lcv.data(), sep ? lcp.data() : nullptr, vl2g.data(), pl2g.data(), nbrs.data(), soff.data(),
                     sd.data(), roff.data(), rd.data()),
       "gls_gpart_get");
    gls_gpart_destroy(gp);
    const int64_t NVD = (int64_t)dim * mm.nv;
    loc.l2g.clear();
    loc.own_l.clear();
    loc.own_g.clear();
    for (int64_t i = 0; i < nvl; ++i)
      for (int c = 0; c < dim; ++c) loc.l2g.push_back(vl2g[(size_t)i] * dim + c);
    for (int64_t j = 0; j < npl; ++j) loc.l2g.push_back(NVD + pl2g[(size_t)j]);
    for (int64_t i = 0; i < nov * dim; ++i) loc.own_l.push_back(i);
    for (int64_t j = 0; j < nop; ++j) loc.own_l.push_back((int64_t)dim * nvl + j);
    for (int64_t i : loc.own_l) loc.own_g.push_back(loc.l2g[(size_t)i]);
    loc.g2l.assign((size_t)mm.n_dofs(), -1);
    for (size_t i = 0; i < loc.l2g.size(); ++i) loc.g2l[(size_t)loc.l2g[i]] = (int64_t)i;
    std::vector<uint8_t> lmask((size_t)nvl);
    for (int64_t i = 0; i < nvl; ++i) lmask[(size_t)i] = cc.mask[(size_t)vl2g[(size_t)i]];
    gls_mesh_desc D;
    std::memset(&D, 0, sizeof(D));
    D.dim = dim;
    D.k = mm.k;
    D.kp = mm.kp;
    D.n_cells = (int)ncl;
    D.n_vnodes = (int)nvl;
    D.n_pnodes = (int)npl;
    D.cell_vnodes = lcv.data();
    D.cell_pnodes = sep ? lcp.data() : nullptr;
    D.map_degree = mm.k;
    D.cell_support = mm.support.data() + (size_t)(cb * nvc * dim);
    D.vnode_mask = lmask.data();
    D.viscosity = P.nu;
    D.srf = P.srf ? 1 : 0;
    for (int i = 0; i < 3; ++i) D.omega[i] = P.omega[i];
    gls_ctx *g = nullptr;
    ck(gls_create(&D, &g), "gls_create");
    if (P.source) {  // forcing at the library's (mapped) quadrature points of the local cells
      const int nq1 = mm.k + 1, nq = dim == 3 ? nq1 * nq1 * nq1 : nq1 * nq1;
      std::vector<double> X((size_t)(ncl * nq * dim)), F, fq(X.size());
      ck(gls_quadrature_points(g, X.data()), "gls_quadrature_points");
      P.force.eval(X, dim, time, F);
      for (size_t i = 0; i < fq.size() / dim; ++i)
        for (int d = 0; d < dim; ++d) fq[i * dim + d] = F[i * (size_t)P.force.nc + d];
      ck(gls_set_force(g, fq.data()), "gls_set_force");
    }
    std::vector<int64_t> dd;
    std::vector<double> dv;
    for (size_t i = 0; i < cc.dofs.size(); ++i) {
      const int64_t l = loc.g2l[(size_t)cc.dofs[i]];
      if (l >= 0) {
        dd.push_back(l);
        dv.push_back(cc.vals[i]);
      }
    }
    ck(gls_set_dirichlet(g, (int64_t)dd.size(), dd.data(), dv.data()), "gls_set_dirichlet");
    if (rccl) {
      ck(gls_dist_attach_dofs_rccl(g, rccl, nov, nop, nn, nbrs.data(), soff.data(), sd.data(), roff.data(), rd.data()),
         "gls_dist_attach_dofs_rccl");
    } else {
      loc.xchg.reset(new ShmExchange);
      ShmExchange &x = *loc.xchg;
      x.nbrs = nbrs;
      x.soff = soff;
      x.roff = roff;
      hk(hipMalloc(&x.send, sizeof(double) * (size_t)std::max<int64_t>(ns, 1)), "hipMalloc");
      hk(hipMalloc(&x.recv, sizeof(double) * (size_t)std::max<int64_t>(nr, 1)), "hipMalloc");
      hk(hipMalloc(&x.red, sizeof(double) * 256), "hipMalloc");
      ck(gls_dist_attach_dofs(g, nov, nop, nn, soff.data(), sd.data(), roff.data(), rd.data(), x.send, x.recv, x.red,
                              ShmExchange::exchange, ShmExchange::allreduce, &x),
         "gls_dist_attach_dofs");
    }
    return g;
  }

  void alloc_vectors() {
    const int64_t N = m.n_dofs(), nd = ndev();
    for (double **q : {&d_present, &d_m1, &d_m2, &d_m3}) {
      hk(hipMalloc(q, sizeof(double) * (size_t)nd), "hipMalloc");
      hk(hipMemset(*q, 0, sizeof(double) * (size_t)nd), "hipMemset");
    }
    present.assign((size_t)N, 0.);
    m1 = m2 = m3 = present;
    dev_ok = true;  // both sides hold zeros
    host_ok = true;
  }
  void need_dev() {  // host -> device (after host-side initial conditions / transfers)
    if (dev_ok) return;
    upload(present, d_present);
    upload(m1, d_m1);
    upload(m2, d_m2);
    upload(m3, d_m3);
    dev_ok = true;
  }
  void need_host() {  // device -> host (output, post-processing, adaptation)
    if (host_ok) return;
    hk(hipDeviceSynchronize(), "need_host");
    download(d_present, present);
    download(d_m1, m1);
    download(d_m2, m2);
    download(d_m3, m3);
    host_ok = true;
  }
  void host_changed() { dev_ok = false; host_ok = true; }
  void dev_changed() { host_ok = false; dev_ok = true; }
  void dcopy(double *dst, const double *src) {  // ordered against the context's own stream: synchronous
    hk(hipDeviceSynchronize(), "device copy");
    hk(hipMemcpy(dst, src, sizeof(double) * (size_t)ndev(), hipMemcpyDeviceToDevice), "device copy");
    hk(hipDeviceSynchronize(), "device copy");
  }

  // node-level hanging lines -> DoF-level lines: velocity DoF node*dim + c per component, pressure
  // DoF dim*nv + node
  static void load_hanging(Mesh &r, int64_t nvh, const int64_t *vn, const int64_t *vo, const int64_t *vm,
                           const double *vw, int64_t nph, const int64_t *pn, const int64_t *po, const int64_t *pm,
                           const double *pw) {
    const int dim = r.dim;
    r.vhanging.assign((size_t)r.nv, 0);
    r.hang_dofs.clear();
    r.hang_off.assign(1, 0);
    r.hang_master.clear();
    r.hang_w.clear();
    for (int64_t i = 0; i < nvh; ++i) {
      r.vhanging[(size_t)vn[i]] = 1;
      for (int c = 0; c < dim; ++c) {
        r.hang_dofs.push_back(vn[i] * dim + c);
        for (int64_t j = vo[i]; j < vo[i + 1]; ++j) {
          r.hang_master.push_back(vm[j] * dim + c);
          r.hang_w.push_back(vw[j]);
        }
        r.hang_off.push_back((int64_t)r.hang_master.size());
      }
    }
    for (int64_t i = 0; i < nph; ++i) {
      r.hang_dofs.push_back(dim * r.nv + pn[i]);
      for (int64_t j = po[i]; j < po[i + 1]; ++j) {
        r.hang_master.push_back(dim * r.nv + pm[j]);
        r.hang_w.push_back(pw[j]);
      }
      r.hang_off.push_back((int64_t)r.hang_master.size());
    }
  }

  // the app's Mesh of a forest mesh (gls_octree_mesh): cells, node maps and coordinates, hanging lines
  Mesh mesh_of_refined(const gls_refined_mesh &R) const {
    const int dim = P.dim;
    const int nvl = dim == 3 ? (P.k + 1) * (P.k + 1) * (P.k + 1) : (P.k + 1) * (P.k + 1);
    const int npl = dim == 3 ? (P.kp + 1) * (P.kp + 1) * (P.kp + 1) : (P.kp + 1) * (P.kp + 1);
    Mesh r;
    r.dim = dim;
    r.n = 1;
    r.k = P.k;
    r.kp = P.kp;
    r.lo = P.lo;
    r.hi = P.hi;
    r.hc = P.hi - P.lo;
    r.nc = R.n_cells;
    r.nv = R.n_vnodes;
    r.np = R.n_pnodes;
    r.cv.assign(R.cell_vnodes, R.cell_vnodes + r.nc * nvl);
    r.cp.assign(R.cell_pnodes, R.cell_pnodes + r.nc * npl);
    r.x0.assign(R.cell_x0, R.cell_x0 + r.nc * dim);
    r.h.assign(R.cell_h, R.cell_h + r.nc * dim);
    r.vx.assign(R.vnode_x, R.vnode_x + r.nv * dim);
    r.px.assign(R.pnode_x, R.pnode_x + r.np * dim);
    load_hanging(r, R.n_vhang, R.vhang_node, R.vhang_off, R.vhang_master, R.vhang_w, R.n_phang, R.phang_node,
                 R.phang_off, R.phang_master, R.phang_w);
    return r;
  }

  // an adapted hyper_cube (gls_octree_mesh, hanging nodes; rmesh already set): mesh, Dirichlet
  // constraints (hanging nodes excluded), hanging constraint lines on the context. Per-cell kernels;
  // one rank, non-periodic, method = amg or --precond hmg: the multigrid V-cycle on the forest's refinement
  // hierarchy (attach_forest_mg; damped-Jacobi smoothing for equal order, ILU(0) smoothing for Q2-Q1), else
  // ILU / Jacobi.
  void setup_refined(gls_refined_mesh *R_new) {
    SectionTimer::Scope ts(timer, "setup_dofs");
    release();
    rmesh = R_new;
    Mesh r = mesh_of_refined(*rmesh);
    r.pmask = m.pmask;  // periodic faces identified by the forest mesh
    m = std::move(r);
    C = make_constraints(P, m, time);
    ctx = make_context(m, C);
    ck(gls_set_hanging(ctx, (int64_t)m.hang_dofs.size(), m.hang_dofs.data(), m.hang_off.data(),
                       m.hang_master.data(), m.hang_w.data()),
       "gls_set_hanging");
    alloc_vectors();
    // as on general meshes: method = amg (ML's hierarchy -> the forest's) or --precond hmg; gmres / bicgstab
    // keep the reference's ILU (setup_ILU, gls_navier_stokes.cc:1161-1176)
    if (use_mg && world == 1 && m.pmask == 0 && tree && ((P.lin_method == 2 && forest_mode != 1) || forest_mode == 2))
      attach_forest_mg();
    print_setup(std::pow(P.hi - P.lo, P.dim));
    std::printf("   Hanging node DoFs:            %lld\n", (long long)m.hang_dofs.size());
  }

  // Geometric multigrid on the forest's refinement hierarchy (gls_mg_attach_transfers): the levels are
  // the forest coarsened one level at a time (gls_octree_coarsen_to) down to 2^dim cells, each with its
  // Dirichlet constraints and hanging lines, the transfers the nested-space interpolation
  // (gls_octree_mg_transfer); FP64 damped-Jacobi V(2,2) at 0.6 (the per-cell levels), exact LU on the
  // coarsest level. The reference preconditions with ILU / ML-AMG (gls_navier_stokes.cc:1161-1240);
  // the substitution is announced (announce_linear_solver).
  std::vector<gls_refined_mesh *> mg_meshes;
  void attach_forest_mg() {
    int L = 0;
    ck(gls_octree_info(tree, nullptr, &L), "gls_octree_info");
    if (L < 2) return;
    std::vector<gls_ctx *> lv{ctx};
    std::vector<const gls_refined_mesh *> meshes{rmesh};
    for (int l = L - 1; l >= 1; --l) {
      gls_octree *tc = nullptr;
      ck(gls_octree_coarsen_to(tree, l, &tc), "gls_octree_coarsen_to");
      gls_refined_mesh *R = nullptr;
      const int rc = gls_octree_mesh(tc, P.k, P.kp, P.lo, P.hi, &R);
      gls_octree_destroy(tc);
      ck(rc, "gls_octree_mesh");
      mg_meshes.push_back(R);
      meshes.push_back(R);
      const Mesh r = mesh_of_refined(*R);
      const Constraints cc = make_constraints(P, r, time);
      gls_ctx *g = make_context(r, cc);
      mg_levels.push_back(g);
      lv.push_back(g);
      if (!r.hang_dofs.empty())
        ck(gls_set_hanging(g, (int64_t)r.hang_dofs.size(), r.hang_dofs.data(), r.hang_off.data(), r.hang_master.data(),
                           r.hang_w.data()),
           "gls_set_hanging (multigrid level)");
    }
    const size_t np = lv.size() - 1;
    std::vector<std::vector<int64_t>> off(np), inj(np);
    std::vector<std::vector<int32_t>> col(np);
    std::vector<std::vector<double>> w(np);
    std::vector<const int64_t *> po(np), pi(np);
    std::vector<const int32_t *> pc(np);
    std::vector<const double *> pw(np);
    for (size_t l = 0; l < np; ++l) {
      int64_t nnz = 0, nf = 0, nco = 0;
      ck(gls_octree_mg_transfer(meshes[l], meshes[l + 1], &nnz, nullptr, nullptr, nullptr, nullptr), "gls_octree_mg_transfer");
      if (l == 0)
        nf = m.n_dofs();  // the fine space's (global) DoFs: with --np, lv[0] is the rank-local context
      else
        ck(gls_n_dofs(lv[l], &nf), "gls_n_dofs");
      ck(gls_n_dofs(lv[l + 1], &nco), "gls_n_dofs");
      off[l].resize((size_t)nf + 1);
      col[l].resize((size_t)std::max<int64_t>(nnz, 1));
      w[l].resize((size_t)std::max<int64_t>(nnz, 1));
      inj[l].resize((size_t)nco);
      ck(gls_octree_mg_transfer(meshes[l], meshes[l + 1], &nnz, off[l].data(), col[l].data(), w[l].data(), inj[l].data()),
         "gls_octree_mg_transfer");
      po[l] = off[l].data();
      pc[l] = col[l].data();
      pw[l] = w[l].data();
      pi[l] = inj[l].data();
    }
    gls_mg_params mp;
    std::memset(&mp, 0, sizeof(mp));
    mp.n_levels = (int)lv.size();
    mp.levels = lv.data();
    mp.smoother = P.k != P.kp ? 1 : 0;  // Q2-Q1: ILU(0) sweeps (point Jacobi sees only the PSPG pressure diagonal)
    mp.pre_smooth = mp.smoother ? 1 : 2;
    mp.post_smooth = mp.smoother ? 1 : 2;
    mp.omega = 0.6;
    mp.coarse_direct = 1;
    ck(gls_mg_attach_transfers(ctx, &mp, po.data(), pc.data(), pw.data(), pi.data()), "gls_mg_attach_transfers");
  }

  void setup(int n) {
    SectionTimer::Scope ts(timer, "setup_dofs");
    release();
    m = build_mesh(P, n, periodic_mask());
    C = make_constraints(P, m, time);
    ctx = make_context(m, C);
    const int64_t N = m.n_dofs();
    alloc_vectors();
    // geometric multigrid on nested hyper_cubes (3D, k == kp <= 2, no periodicity)
    if (use_mg && P.dim == 3 && P.k == P.kp && P.k <= 2 && m.pmask == 0 && n >= 4 && (n & (n - 1)) == 0) {
      std::vector<gls_ctx *> lv{ctx};
      for (int c = n / 2; c >= 2; c /= 2) {
        const Mesh mc = build_mesh(P, c, 0);
        const Constraints cc = make_constraints(P, mc, time);
        gls_ctx *g = make_context(mc, cc);
        mg_levels.push_back(g);
        lv.push_back(g);
      }
      gls_mg_params mp;
      std::memset(&mp, 0, sizeof(mp));
      mp.n_levels = (int)lv.size();
      mp.levels = lv.data();
      mp.pre_smooth = 1;
      mp.post_smooth = 1;
      mp.coarse_sweeps = 100;
      mp.omega = 0.9;
      mp.coarse_omega = 0.7;
      mp.mixed_precision = 1;    // FP32 smoothing J.v (the outer GMRES operator stays the FP64 Jacobian)
      mp.smoother_operator = 1;  // ... with the Oseen (Picard) linearization (bench.py's V-cycle)
      ck(gls_mg_attach(ctx, &mp), "gls_mg_attach");
    }
    (void)N;
    print_setup(std::pow(P.hi - P.lo, P.dim));
  }

  // general meshes: the triangulation (gmsh file or GridGenerator grid with its manifolds and the
  // prm's spherical boundary manifolds, refine_global(initial refinement)), read once
  void create_umesh() {
    if (P.mesh_type == "gmsh") ck(gls_umesh_read_gmsh(P.dim, P.mesh_file.c_str(), &um), "reading the gmsh mesh");
    else ck(gls_umesh_generate(P.dim, P.grid_type.c_str(), P.grid_args.c_str(), &um), "GridGenerator");
    for (const auto &mp : P.manifolds) {  // attach_manifolds_to_triangulation (manifolds.cc:226-247)
      if (mp.type != "spherical") continue;
      ck(gls_umesh_set_manifold(um, mp.id, 1, mp.arg, nullptr), "gls_umesh_set_manifold");
      ck(gls_umesh_boundary_manifold(um, mp.id, mp.id), "gls_umesh_boundary_manifold");
    }
    // periodic pairs of the triangulation (attach_grid_to_triangulation's add_periodicity, grids.cc:41-58):
    // the Kelly adaptation keeps the levels across them within one of each other
    std::vector<int32_t> per;
    for (const BC &b : P.bcs)
      if (b.type == "periodic") {
        per.push_back(b.id);
        per.push_back(b.periodic_id);
        per.push_back(b.periodic_direction);
      }
    if (!per.empty()) ck(gls_umesh_set_periodic(um, (int)per.size() / 3, per.data()), "gls_umesh_set_periodic");
    ck(gls_umesh_refine_global(um, P.refinement), "refine_global");
  }
  // the app's Mesh of an FE space of the triangulation (cells, nodes, MappingQ support points, hanging
  // lines, the slip boundaries' averaged node normals)
  Mesh mesh_of_space(const gls_fe_space &F, int k = -1, int kp = -1) {  // k, kp: the space's degrees (P's default)
    k = k < 0 ? P.k : k;
    kp = kp < 0 ? P.kp : kp;
    Mesh r;
    r.dim = P.dim;
    r.k = k;
    r.kp = kp;
    r.general = true;
    r.nc = F.n_cells;
    r.nv = F.n_vnodes;
    r.np = F.n_pnodes;
    const int nvl = P.dim == 3 ? (k + 1) * (k + 1) * (k + 1) : (k + 1) * (k + 1);
    const int npl = P.dim == 3 ? (kp + 1) * (kp + 1) * (kp + 1) : (kp + 1) * (kp + 1);
    r.cv.assign(F.cell_vnodes, F.cell_vnodes + r.nc * nvl);
    r.cp.assign(F.cell_pnodes, F.cell_pnodes + r.nc * npl);
    r.vx.assign(F.vnode_x, F.vnode_x + r.nv * P.dim);
    r.px.assign(F.pnode_x, F.pnode_x + r.np * P.dim);
    r.vbid.assign(F.vnode_bid, F.vnode_bid + r.nv);
    r.support.assign(F.cell_support, F.cell_support + r.nc * nvl * P.dim);
    r.measure.assign(F.cell_measure, F.cell_measure + r.nc);
    load_hanging(r, F.n_vhang, F.vhang_node, F.vhang_off, F.vhang_master, F.vhang_w, F.n_phang, F.phang_node,
                 F.phang_off, F.phang_master, F.phang_w);
    // slip boundaries: the averaged face normals at the velocity nodes (compute_no_normal_flux_constraints)
    for (const BC &b : P.bcs)
      if (b.type == "slip") {
        std::vector<double> nrm((size_t)(r.nv * P.dim)), sets((size_t)(r.nv * 3 * P.dim));
        std::vector<int32_t> rank_((size_t)r.nv);
        ck(gls_fe_space_boundary_normals(&F, b.id, nrm.data()), "gls_fe_space_boundary_normals");
        ck(gls_fe_space_boundary_normal_sets(&F, b.id, rank_.data(), sets.data()), "gls_fe_space_boundary_normal_sets");
        r.slip_normals[b.id] = std::move(nrm);
        r.slip_rank[b.id] = std::move(rank_);
        r.slip_sets[b.id] = std::move(sets);
      }
    return r;
  }
  // the context's constraint lines: hanging lines + slip lines of curved walls, chains closed
  void constraint_lines(const Mesh &mm, const Constraints &cc, std::vector<int64_t> &ld, std::vector<int64_t> &lo,
                        std::vector<int64_t> &lm, std::vector<double> &lw) {
    ld = mm.hang_dofs;
    lo = mm.hang_off;
    lm = mm.hang_master;
    lw = mm.hang_w;
    for (size_t i = 0; i < cc.line_dofs.size(); ++i) {
      ld.push_back(cc.line_dofs[i]);
      for (int64_t j = cc.line_off[i]; j < cc.line_off[i + 1]; ++j) {
        lm.push_back(cc.line_master[(size_t)j]);
        lw.push_back(cc.line_w[(size_t)j]);
      }
      lo.push_back((int64_t)lm.size());
    }
    close_lines(ld, lo, lm, lw);
  }

  // Geometric multigrid on the triangulation's refinement hierarchy (gls_mg_attach_transfers): levels =
  // the triangulation coarsened one level at a time (gls_umesh_coarsen_to) down to the coarse mesh, each
  // with its FE space, MappingQ geometry, Dirichlet / slip constraints and hanging lines; transfers =
  // FE_Q's embedding (gls_fe_space_mg_transfer); FP64 damped-Jacobi V(2,2) at 0.6, exact LU on the
  // coarsest level when it is small enough (<= 8192 DoFs), else 30 Jacobi sweeps there. Q2-Q1 / Q2-Q2: below the
  // base mesh a p-level -- Q1-Q1 on the base mesh's cells (gls_fe_space_mg_transfer's p-level pair), factored by
  // the dense LU (<= kPLevelDirectMax DoFs) -- whenever the base level is too large for the LU itself; this is also
  // the whole hierarchy of an unrefined mesh (the reference's setup_AMG, gls_navier_stokes.cc:1180-1240: an
  // algebraic multilevel preconditioner there, a geometric / polynomial one here, announced on stderr).
  static constexpr int64_t kPLevelDirectMax = 40000;
  bool plevel_used = false;
  void attach_umesh_mg() {
    int L = 0;
    for (int64_t c = 0; c < space->n_cells; ++c) L = std::max(L, (int)space->cell_level[c]);
    plevel_used = false;
    if (L < 1 && P.k < 2) return;
    std::vector<gls_ctx *> lv{ctx};
    std::vector<gls_fe_space *> spaces;
    std::vector<const gls_fe_space *> sp{space};
    int64_t n_coarse = 0;
    for (int l = L - 1; l >= 0; --l) {
      gls_umesh *uc = nullptr;
      ck(gls_umesh_coarsen_to(um, l, &uc), "gls_umesh_coarsen_to");
      gls_fe_space *s_ = nullptr;
      const int rc = gls_umesh_fe_space(uc, P.k, P.kp, P.qmapping_all ? 1 : 0, 0, nullptr, &s_);
      gls_umesh_destroy(uc);
      ck(rc, "gls_umesh_fe_space (multigrid level)");
      spaces.push_back(s_);
      sp.push_back(s_);
      const Mesh r = mesh_of_space(*s_);
      const Constraints cc = make_constraints(P, r, time);
      std::vector<int64_t> ld, lo, lm;
      std::vector<double> lw;
      constraint_lines(r, cc, ld, lo, lm, lw);
      gls_ctx *g = make_context(r, cc);
      mg_levels.push_back(g);
      lv.push_back(g);
      if (!ld.empty()) ck(gls_set_hanging(g, (int64_t)ld.size(), ld.data(), lo.data(), lm.data(), lw.data()), "gls_set_hanging (multigrid level)");
      n_coarse = r.n_dofs();
    }
    if (P.k >= 2 && (L < 1 || n_coarse > 8192)) {  // the Q1-Q1 p-level on the base mesh
      gls_umesh *uc = nullptr;
      ck(gls_umesh_coarsen_to(um, 0, &uc), "gls_umesh_coarsen_to");
      gls_fe_space *s_ = nullptr;
      const int rc = gls_umesh_fe_space(uc, 1, 1, P.qmapping_all ? 1 : 0, 0, nullptr, &s_);
      gls_umesh_destroy(uc);
      ck(rc, "gls_umesh_fe_space (p-level)");
      const Mesh r = mesh_of_space(*s_, 1, 1);
      if (r.n_dofs() <= kPLevelDirectMax) {
        spaces.push_back(s_);
        sp.push_back(s_);
        const Constraints cc = make_constraints(P, r, time);
        std::vector<int64_t> ld, lo, lm;
        std::vector<double> lw;
        constraint_lines(r, cc, ld, lo, lm, lw);
        gls_ctx *g = make_context(r, cc);
        mg_levels.push_back(g);
        lv.push_back(g);
        if (!ld.empty()) ck(gls_set_hanging(g, (int64_t)ld.size(), ld.data(), lo.data(), lm.data(), lw.data()), "gls_set_hanging (p-level)");
        n_coarse = r.n_dofs();
        plevel_used = true;
      } else {
        gls_fe_space_destroy(s_);
      }
    }
    if (lv.size() < 2) return;
    const size_t np = lv.size() - 1;
    std::vector<std::vector<int64_t>> off(np), inj(np);
    std::vector<std::vector<int32_t>> col(np);
    std::vector<std::vector<double>> w(np);
    std::vector<const int64_t *> po(np), pi(np);
    std::vector<const int32_t *> pc(np);
    std::vector<const double *> pw(np);
    for (size_t l = 0; l < np; ++l) {
      int64_t nnz = 0, nf = 0, nco = 0;
      ck(gls_fe_space_mg_transfer(sp[l], sp[l + 1], &nnz, nullptr, nullptr, nullptr, nullptr), "gls_fe_space_mg_transfer");
      if (l == 0)
        nf = m.n_dofs();  // the fine space's (global) DoFs: with --np, lv[0] is the rank-local context
      else
        ck(gls_n_dofs(lv[l], &nf), "gls_n_dofs");
      ck(gls_n_dofs(lv[l + 1], &nco), "gls_n_dofs");
      off[l].resize((size_t)nf + 1);
      col[l].resize((size_t)std::max<int64_t>(nnz, 1));
      w[l].resize((size_t)std::max<int64_t>(nnz, 1));
      inj[l].resize((size_t)nco);
      ck(gls_fe_space_mg_transfer(sp[l], sp[l + 1], &nnz, off[l].data(), col[l].data(), w[l].data(), inj[l].data()),
         "gls_fe_space_mg_transfer");
      po[l] = off[l].data();
      pc[l] = col[l].data();
      pw[l] = w[l].data();
      pi[l] = inj[l].data();
    }
    for (gls_fe_space *s_ : spaces) gls_fe_space_destroy(s_);
    gls_mg_params mp;
    std::memset(&mp, 0, sizeof(mp));
    mp.n_levels = (int)lv.size();
    mp.levels = lv.data();
    mp.smoother = P.k != P.kp ? 1 : 0;  // Q2-Q1: ILU(0) sweeps (point Jacobi sees only the PSPG pressure diagonal)
    mp.pre_smooth = mp.smoother ? 1 : 2;
    mp.post_smooth = mp.smoother ? 1 : 2;
    mp.omega = 0.6;
    mp.coarse_direct = n_coarse <= (plevel_used ? kPLevelDirectMax : 8192) ? 1 : -1;
    if (world == 1) {
      ck(gls_mg_attach_transfers(ctx, &mp, po.data(), pc.data(), pw.data(), pi.data()), "gls_mg_attach_transfers");
      return;
    }
    // --np: the fine level is this rank's cells; levels 1..L (whole meshes) run on every rank as one replica
    // hierarchy fed by the all-reduced restriction of the owned rows (gls_mg_attach_replica). P's rows of the
    // rank's local fine DoFs; a level-1 DoF's state comes from the fine DoF it injects, on the rank owning it.
    gls_ctx *replica = lv[1];
    if (lv.size() > 2) {
      gls_mg_params rp = mp;
      rp.n_levels = (int)lv.size() - 1;
      rp.levels = lv.data() + 1;
      ck(gls_mg_attach_transfers(replica, &rp, po.data() + 1, pc.data() + 1, pw.data() + 1, pi.data() + 1),
         "gls_mg_attach_transfers (replica)");
    }
    std::vector<int64_t> loff{0};
    std::vector<int32_t> lcol;
    std::vector<double> lwt;
    for (int64_t g : loc.l2g) {
      for (int64_t j = off[0][(size_t)g]; j < off[0][(size_t)g + 1]; ++j) {
        lcol.push_back(col[0][(size_t)j]);
        lwt.push_back(w[0][(size_t)j]);
      }
      loff.push_back((int64_t)lcol.size());
    }
    std::vector<uint8_t> owned(loc.l2g.size(), 0);
    for (int64_t i : loc.own_l) owned[(size_t)i] = 1;
    std::vector<int64_t> linj(inj[0].size(), -1);
    for (size_t j = 0; j < inj[0].size(); ++j) {
      const int64_t l = loc.g2l[(size_t)inj[0][j]];
      if (l >= 0 && owned[(size_t)l]) linj[j] = l;
    }
    if (lcol.empty()) lcol.push_back(0), lwt.push_back(0.0);
    gls_mg_params fp = mp;
    fp.n_levels = 1;
    fp.levels = lv.data();
    ck(gls_mg_attach_replica(ctx, &fp, replica, loff.data(), lcol.data(), lwt.data(), linj.data()), "gls_mg_attach_replica");
  }

  // FE space, constraints and context on the current triangulation (per-cell kernels with MappingQ
  // geometry, Jacobi-preconditioned GMRES)
  void setup_general() {
    SectionTimer::Scope ts(timer, "setup_dofs");
    release();
    if (space) gls_fe_space_destroy(space);
    space = nullptr;
    std::vector<int32_t> per;
    for (const BC &b : P.bcs)
      if (b.type == "periodic") {  // make_periodicity_constraints(id, periodic_id, direction)
        per.push_back(b.id);
        per.push_back(b.periodic_id);
        per.push_back(b.periodic_direction);
      }
    ck(gls_umesh_fe_space(um, P.k, P.kp, P.qmapping_all ? 1 : 0, (int)per.size() / 3, per.data(), &space), "gls_umesh_fe_space");
    const gls_fe_space &F = *space;
    m = mesh_of_space(F);
    if (!per.empty()) {  // deal.II's DoF count: the same space without the periodic identification
      gls_fe_space *raw = nullptr;
      ck(gls_umesh_fe_space(um, P.k, P.kp, P.qmapping_all ? 1 : 0, 0, nullptr, &raw), "gls_umesh_fe_space");
      m.n_dofs_dealii = (int64_t)P.dim * raw->n_vnodes + raw->n_pnodes;
      gls_fe_space_destroy(raw);
    }
    C = make_constraints(P, m, time);
    // hanging lines + slip lines of curved walls (homogeneous constraint lines on velocity DoFs)
    std::vector<int64_t> ld, lo, lm;
    std::vector<double> lw;
    constraint_lines(m, C, ld, lo, lm, lw);
    g_lines = {ld, lo, lm};
    g_lines_w = lw;
    if (world > 1) {  // the rank's cells; its lines in local DoF ids (masters are local by construction)
      ctx = make_context_local(m, C, ld, lo, lm);
      std::vector<int64_t> ld2, lo2{0}, lm2;
      std::vector<double> lw2;
      for (size_t i = 0; i < ld.size(); ++i) {
        const int64_t l = loc.g2l[(size_t)ld[i]];
        if (l < 0) continue;
        ld2.push_back(l);
        for (int64_t j = lo[i]; j < lo[i + 1]; ++j) {
          const int64_t mj = loc.g2l[(size_t)lm[(size_t)j]];
          if (mj < 0) die("rank %d: a line master is not local", rank);
          lm2.push_back(mj);
          lw2.push_back(lw[(size_t)j]);
        }
        lo2.push_back((int64_t)lm2.size());
      }
      if (!ld2.empty())
        ck(gls_set_hanging(ctx, (int64_t)ld2.size(), ld2.data(), lo2.data(), lm2.data(), lw2.data()), "gls_set_hanging");
      // --precond hmg (or method = amg): the one-rank V-cycle with a replicated coarse hierarchy
      if (use_mg && per.empty() && ((P.lin_method == 2 && forest_mode != 1) || forest_mode == 2))
        attach_umesh_mg();
    } else {
      ctx = make_context(m, C);
      if (!ld.empty())
        ck(gls_set_hanging(ctx, (int64_t)ld.size(), ld.data(), lo.data(), lm.data(), lw.data()), "gls_set_hanging");
      // method = amg (ML's multilevel hierarchy): the geometric one of the triangulation, every order (Q2-Q1
      // levels smooth with multicolor ILU(0), equal order with damped Jacobi); gmres keeps the reference's ILU
      // (--precond hmg: the hierarchy multigrid for every method)
      if (use_mg && per.empty() && ((P.lin_method == 2 && forest_mode != 1) || forest_mode == 2))
        attach_umesh_mg();
    }
    alloc_vectors();
    print_setup(F.volume);
  }
  // setup_dofs' summary lines (gls_navier_stokes.cc:220-227)
  void print_setup(double volume) {
    std::printf("   Number of active cells:       %lld\n   Number of degrees of freedom: %lld\n", (long long)m.nc,
                (long long)(m.n_dofs_dealii >= 0 ? m.n_dofs_dealii : m.n_dofs()));
    std::printf("   Volume of triangulation:      %g\n", volume);
  }

  void upload(const std::vector<double> &h, double *d) {  // global host vector -> (rank-local) device vector
    if (world > 1) {
      loc.tmp.resize(loc.l2g.size());
      for (size_t i = 0; i < loc.l2g.size(); ++i) loc.tmp[i] = h[(size_t)loc.l2g[i]];
      hk(hipMemcpy(d, loc.tmp.data(), sizeof(double) * loc.tmp.size(), hipMemcpyHostToDevice), "upload");
      return;
    }
    hk(hipMemcpy(d, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice), "upload");
  }
  void download(const double *d, std::vector<double> &h) {  // --np: every rank's owned values, gathered
    if (world > 1) {
      loc.tmp.resize(loc.l2g.size());
      hk(hipMemcpy(loc.tmp.data(), d, sizeof(double) * loc.tmp.size(), hipMemcpyDeviceToHost), "download");
      std::vector<double> own(loc.own_l.size());
      for (size_t i = 0; i < own.size(); ++i) own[i] = loc.tmp[(size_t)loc.own_l[i]];
      g_comm.allgather(own.data(), loc.own_g, h);
      return;
    }
    hk(hipMemcpy(h.data(), d, sizeof(double) * h.size(), hipMemcpyDeviceToHost), "download");
  }

  // ---- initial conditions
  void nodal_values(const Function &f, std::vector<double> &x) {  // interpolation + Dirichlet values
    for (int part = 0; part < 2; ++part) {
      const bool vel = part == 0;
      const int64_t nn = vel ? m.nv : m.np;
      std::vector<double> X, F;
      for (int64_t v = 0; v < nn; ++v) {
        double c[3];
        int idx[3];
        m.coord(v, vel, c, idx);
        X.insert(X.end(), c, c + m.dim);
      }
      f.eval(X, m.dim, time, F);
      for (int64_t v = 0; v < nn; ++v) {
        if (vel)
          for (int d = 0; d < m.dim; ++d) x[(size_t)(v * m.dim + d)] = F[(size_t)(v * f.nc + d)];
        else
          x[(size_t)(m.dim * m.nv + v)] = F[(size_t)(v * f.nc + m.dim)];
      }
    }
    for (size_t i = 0; i < C.dofs.size(); ++i) x[(size_t)C.dofs[i]] = C.vals[i];
  }

  // L2 projection of uvwp onto the velocity-pressure space: consistent mass matrix (block diagonal
  // per component), host conjugate gradients to 1e-15 relative; Dirichlet rows keep their values
  void l2_projection(const Function &f, std::vector<double> &x) {
    const int nq1 = m.k + 1, dim = m.dim;
    CellEval ev(m, nq1);
    const int64_t N = m.n_dofs(), voff = (int64_t)dim * m.nv;
    std::vector<double> X, F, rhs((size_t)N, 0.0), wq((size_t)(m.nc * ev.nq));
    for (int64_t c = 0; c < m.nc; ++c)
      for (int q = 0; q < ev.nq; ++q) {
        double xx[3], w;
        ev.point(c, q, xx, w);
        wq[(size_t)(c * ev.nq + q)] = w;
        X.insert(X.end(), xx, xx + dim);
      }
    f.eval(X, dim, time, F);
    for (int64_t c = 0; c < m.nc; ++c)
      for (int q = 0; q < ev.nq; ++q) {
        int qq[3];
        ev.qidx(q, qq);
        const double w = wq[(size_t)(c * ev.nq + q)];
        const double *fv = &F[(size_t)((c * ev.nq + q) * f.nc)];
        for (int a = 0; a < ev.nvl; ++a) {
          const double ph = ev.phi_v(a, qq) * w;
          for (int d = 0; d < dim; ++d) rhs[(size_t)(m.cv[(size_t)(c * ev.nvl + a)] * dim + d)] += ph * fv[d];
        }
        for (int a = 0; a < ev.npl; ++a) rhs[(size_t)(voff + m.cp[(size_t)(c * ev.npl + a)])] += ev.phi_p(a, qq) * w * fv[dim];
      }
    std::vector<char> fixed((size_t)N, 0);
    for (size_t i = 0; i < C.dofs.size(); ++i) fixed[(size_t)C.dofs[i]] = 1;
    auto mass = [&](const std::vector<double> &in, std::vector<double> &out) {
      std::fill(out.begin(), out.end(), 0.0);
      for (int64_t c = 0; c < m.nc; ++c)
        for (int q = 0; q < ev.nq; ++q) {
          int qq[3];
          ev.qidx(q, qq);
          const double w = wq[(size_t)(c * ev.nq + q)];
          double uq[3] = {0, 0, 0}, pq = 0;
          for (int a = 0; a < ev.nvl; ++a) {
            const double ph = ev.phi_v(a, qq);
            for (int d = 0; d < dim; ++d) uq[d] += ph * in[(size_t)(m.cv[(size_t)(c * ev.nvl + a)] * dim + d)];
          }
          for (int a = 0; a < ev.npl; ++a) pq += ev.phi_p(a, qq) * in[(size_t)(voff + m.cp[(size_t)(c * ev.npl + a)])];
          for (int a = 0; a < ev.nvl; ++a) {
            const double ph = ev.phi_v(a, qq) * w;
            for (int d = 0; d < dim; ++d) out[(size_t)(m.cv[(size_t)(c * ev.nvl + a)] * dim + d)] += ph * uq[d];
          }
          for (int a = 0; a < ev.npl; ++a) out[(size_t)(voff + m.cp[(size_t)(c * ev.npl + a)])] += ev.phi_p(a, qq) * w * pq;
        }
    };
    std::fill(x.begin(), x.end(), 0.0);
    for (size_t i = 0; i < C.dofs.size(); ++i) x[(size_t)C.dofs[i]] = C.vals[i];
    std::vector<double> r((size_t)N), pd((size_t)N), Ap((size_t)N);
    mass(x, Ap);
    double rr = 0, bb = 0;
    for (int64_t i = 0; i < N; ++i) {
      r[(size_t)i] = fixed[(size_t)i] ? 0.0 : rhs[(size_t)i] - Ap[(size_t)i];
      rr += r[(size_t)i] * r[(size_t)i];
      bb += rhs[(size_t)i] * rhs[(size_t)i];
    }
    pd = r;
    for (int it = 0; it < 10000 && rr > 1e-30 * std::max(bb, 1e-300); ++it) {
      mass(pd, Ap);
      double pAp = 0;
      for (int64_t i = 0; i < N; ++i) {
        if (fixed[(size_t)i]) Ap[(size_t)i] = 0.0;
        pAp += pd[(size_t)i] * Ap[(size_t)i];
      }
      const double alpha = rr / pAp;
      double rr2 = 0;
      for (int64_t i = 0; i < N; ++i) {
        x[(size_t)i] += alpha * pd[(size_t)i];
        r[(size_t)i] -= alpha * Ap[(size_t)i];
        rr2 += r[(size_t)i] * r[(size_t)i];
      }
      const double beta = rr2 / rr;
      rr = rr2;
      for (int64_t i = 0; i < N; ++i) pd[(size_t)i] = r[(size_t)i] + beta * pd[(size_t)i];
    }
  }

  // --np diagnostics (GLS_NP_CHECK): the gathered distributed residual at the current state against
  // the residual of a whole-mesh context on rank 0; the largest differences are printed to stderr
  void check_distributed_residual(const double ts[4]) {
    const int64_t N = m.n_dofs(), nd = ndev();
    double *d_r = nullptr;
    hk(hipMalloc(&d_r, sizeof(double) * (size_t)nd), "hipMalloc");
    ck(gls_set_state(ctx, d_present, d_m1, d_m2, d_m3), "gls_set_state");
    ck(gls_residual(ctx, d_r), "gls_residual");
    hk(hipDeviceSynchronize(), "residual");
    std::vector<double> rd((size_t)N), x((size_t)N), h1((size_t)N), h2((size_t)N), h3((size_t)N), vv((size_t)N),
        jd((size_t)N);
    download(d_r, rd);
    for (int64_t i = 0; i < N; ++i) vv[(size_t)i] = std::sin(0.37 * (double)i + 0.1) + 0.5 * std::cos(1.3 * (double)i);
    {
      double *d_v = nullptr, *d_j = nullptr;
      hk(hipMalloc(&d_v, sizeof(double) * (size_t)nd), "hipMalloc");
      hk(hipMalloc(&d_j, sizeof(double) * (size_t)nd), "hipMalloc");
      upload(vv, d_v);
      ck(gls_jacobian_apply(ctx, d_v, d_j), "gls_jacobian_apply");
      hk(hipDeviceSynchronize(), "jv");
      download(d_j, jd);
      (void)hipFree(d_v);
      (void)hipFree(d_j);
    }
    download(d_present, x);
    download(d_m1, h1);
    download(d_m2, h2);
    download(d_m3, h3);
    (void)hipFree(d_r);
    if (rank != 0) return;
    gls_ctx *g = make_context(m, C);
    if (!g_lines[0].empty())
      ck(gls_set_hanging(g, (int64_t)g_lines[0].size(), g_lines[0].data(), g_lines[1].data(), g_lines[2].data(),
                         g_lines_w.data()),
         "gls_set_hanging");
    ck(gls_set_time(g, last_scheme, ts), "gls_set_time");
    double *dv[6];
    for (double *&q : dv) hk(hipMalloc(&q, sizeof(double) * (size_t)N), "hipMalloc");
    const std::vector<double> *hv[4] = {&x, &h1, &h2, &h3};
    for (int i = 0; i < 4; ++i) hk(hipMemcpy(dv[i], hv[i]->data(), sizeof(double) * (size_t)N, hipMemcpyHostToDevice), "upload");
    ck(gls_set_state(g, dv[0], dv[1], dv[2], dv[3]), "gls_set_state");
    ck(gls_residual(g, dv[4]), "gls_residual");
    hk(hipDeviceSynchronize(), "residual");
    std::vector<double> rg((size_t)N), jg((size_t)N);
    hk(hipMemcpy(rg.data(), dv[4], sizeof(double) * (size_t)N, hipMemcpyDeviceToHost), "download");
    hk(hipMemcpy(dv[5], vv.data(), sizeof(double) * (size_t)N, hipMemcpyHostToDevice), "upload");
    ck(gls_jacobian_apply(g, dv[5], dv[4]), "gls_jacobian_apply");
    hk(hipDeviceSynchronize(), "jv");
    hk(hipMemcpy(jg.data(), dv[4], sizeof(double) * (size_t)N, hipMemcpyDeviceToHost), "download");
    {
      double dj = 0, nj = 0;
      int64_t worst = 0;
      for (int64_t i = 0; i < N; ++i) {
        nj += jg[(size_t)i] * jg[(size_t)i];
        const double e = std::fabs(jd[(size_t)i] - jg[(size_t)i]);
        dj += e * e;
        if (e > std::fabs(jd[(size_t)worst] - jg[(size_t)worst])) worst = i;
      }
      std::fprintf(stderr, "np-check: |Jv| %.6e |Jv_dist - Jv| %.6e worst dof %lld dist %.6e whole %.6e\n", std::sqrt(nj),
                   std::sqrt(dj), (long long)worst, jd[(size_t)worst], jg[(size_t)worst]);
    }
    for (double *q : dv) (void)hipFree(q);
    gls_destroy(g);
    std::vector<int64_t> idx((size_t)N);
    double nr = 0, nd2 = 0, ps = 0, psg = 0;
    const int64_t nvd = (int64_t)m.dim * m.nv;
    for (int64_t i = 0; i < N; ++i) {
      idx[(size_t)i] = i;
      nr += rg[(size_t)i] * rg[(size_t)i];
      nd2 += (rd[(size_t)i] - rg[(size_t)i]) * (rd[(size_t)i] - rg[(size_t)i]);
      if (i >= nvd) { ps += rd[(size_t)i]; psg += rg[(size_t)i]; }
    }
    std::partial_sort(idx.begin(), idx.begin() + std::min<int64_t>(N, 8), idx.end(), [&](int64_t a, int64_t b) {
      return std::fabs(rd[(size_t)a] - rg[(size_t)a]) > std::fabs(rd[(size_t)b] - rg[(size_t)b]);
    });
    std::fprintf(stderr, "np-check: |r| %.6e |r_dist - r| %.6e  sum r_p: dist %.6e whole %.6e\n", std::sqrt(nr),
                 std::sqrt(nd2), ps, psg);
    std::vector<char> isline((size_t)N, 0);
    for (int64_t d : g_lines[0]) isline[(size_t)d] = 1;
    for (int t = 0; t < std::min<int64_t>(N, 8); ++t) {
      const int64_t i = idx[(size_t)t];
      const bool vel = i < nvd;
      const int64_t node = vel ? i / m.dim : i - nvd;
      std::fprintf(stderr, "  dof %lld (%s node %lld%s%s) dist %.6e whole %.6e\n", (long long)i, vel ? "u" : "p",
                   (long long)node, isline[(size_t)i] ? ", line" : "",
                   vel && ((C.mask[(size_t)node] >> (i % m.dim)) & 1) ? ", dirichlet" : "", rd[(size_t)i], rg[(size_t)i]);
    }
  }

  // the linear solver and preconditioner actually used for the prm's 'linear solver/method', once per
  // run on stderr (stdout stays the reference's): the substitutions are explicit, never silent
  std::string lin_announced;  // the last announcement (a new one when the preconditioner changes)
  void announce_linear_solver() {
    if (rank != 0) return;
    const char *meth[3] = {"gmres", "bicgstab", "amg"};
    const char *krylov = P.lin_method == 1 ? "BiCGStab" : "GMRES";
    char prec[256];
    if (!mg_levels.empty() && (rmesh || space))
      std::snprintf(prec, sizeof prec, "geometric multigrid %s on the %s refinement hierarchy (%zu levels%s)",
                    P.k != P.kp ? "V(1,1)-cycle with ILU(0) smoothing" : "V(2,2)-cycle with damped-Jacobi smoothing",
                    rmesh ? "forest's" : "triangulation's", mg_levels.size() + 1,
                    plevel_used ? ", the last a Q1-Q1 p-level on the base mesh, dense LU" : "");
    else if (!mg_levels.empty())
      std::snprintf(prec, sizeof prec, "geometric multigrid V(1,1)-cycle on the nested hyper_cubes");
    else if (use_ilu && P.lin_method == 2)
      std::snprintf(prec, sizeof prec, "ILU(%d) atol %g rtol %g (the amg smoother's ILU on the fine level)",
                    P.amg_ilu_fill, P.amg_ilu_atol, P.amg_ilu_rtol);
    else if (use_ilu)
      std::snprintf(prec, sizeof prec, "ILU(%d) atol %g rtol %g", P.ilu_fill, P.ilu_atol, P.ilu_rtol);
    else
      std::snprintf(prec, sizeof prec, "Jacobi (--precond jacobi)");
    char line[512];
    std::snprintf(line, sizeof line, "linear solver: method = %s -> %s + %s%s\n", meth[P.lin_method], krylov, prec,
                  P.lin_method == 2 ? (P.amg_w_cycles ? "; ML AMG substituted (amg w cycles = true: V-cycle used)"
                                                      : "; ML AMG substituted")
                                    : "");
    if (lin_announced == line) return;
    lin_announced = line;
    std::fputs(line, stderr);
  }

  // ---- one nonlinear solve of `scheme` from the current present solution and history
  // solve_non_linear_system(method, first_iteration = false, force_matrix_renewal)
  void solve_nonlinear(int scheme, double nu_override = -1.0, bool force_renewal = false) {
    double ts[4];
    for (int i = 0; i < 4; ++i) ts[i] = dts[i] > 0 ? dts[i] : 1.0;
    ck(gls_set_time(ctx, scheme, ts), "gls_set_time");
    last_scheme = scheme;
    for (int i = 0; i < 4; ++i) last_ts[i] = ts[i];
    if (nu_override > 0) ck(gls_set_viscosity(ctx, nu_override), "gls_set_viscosity");
    need_dev();
    ck(gls_apply_dirichlet(ctx, d_present), "gls_apply_dirichlet");
    if (world > 1 && std::getenv("GLS_NP_CHECK")) check_distributed_residual(ts);
    gls_newton_params np;
    std::memset(&np, 0, sizeof(np));
    np.tolerance = P.newton_tol;
    np.max_iterations = P.newton_max;
    np.verbosity = P.newton_verbose;
    // Preconditioner: the multigrid V-cycle on nested hyper_cubes; elsewhere the reference's
    // ILU(fill)-GMRES (setup_ILU, gls_navier_stokes.cc:1161-1176) with the prm's restart (30, the
    // TrilinosWrappers::SolverGMRES default) and iteration cap, unless --precond jacobi. Jacobi is much
    // weaker than the reference's preconditioners, so its caps and restart are raised.
    if (mg_levels.empty() && use_ilu && ilu_ctx != ctx) {
      // ordering: Cuthill-McKee as the reference factors; above kIluMulticolorDofs, and across ranks
      // (where the block-Jacobi ILU does not reproduce the single-rank iteration counts anyway), the
      // multicolor order, whose triangular solves are ~60x faster on the GPU
      // (profiles/r03_app_cylinder3d_ilu_timing.log vs r03_app_cylinder3d_multicolor_ilu.log) at the price of more GMRES iterations (--ilu-order overrides)
      const int order = ilu_order >= 0 ? ilu_order
                        : (m.n_dofs() > kIluMulticolorDofs || world > 1 ? GLS_ILU_ORDER_MULTICOLOR : GLS_ILU_ORDER_CM);
      ck(gls_ilu_set_options(ctx, order, ilu_block_dofs), "gls_ilu_set_options");
      if (P.lin_method == 2)  // amg: the ILU ML would smooth / coarsen with (setup_AMG, :1225-1233)
        ck(gls_ilu_attach(ctx, P.amg_ilu_fill, P.amg_ilu_atol, P.amg_ilu_rtol), "gls_ilu_attach");
      else
        ck(gls_ilu_attach(ctx, P.ilu_fill, P.ilu_atol, P.ilu_rtol), "gls_ilu_attach");
      ilu_ctx = ctx;
    }
    announce_linear_solver();
    const bool jacobi = mg_levels.empty() && !use_ilu;
    np.lin.max_iterations = jacobi ? std::max(P.lin_max, 20000) : P.lin_max;
    np.lin.restart = jacobi ? std::max(P.restart, 100) : P.restart;
    np.lin.relative_residual = P.lin_rel;
    np.lin.minimum_residual = P.lin_min;
    np.lin.method = P.lin_method == 1 ? GLS_LIN_BICGSTAB : GLS_LIN_GMRES;
    np.solver = P.nl_solver;
    np.skip_iterations = P.skip_iterations;
    np.is_initial_step = 0;
    np.force_matrix_renewal = force_renewal ? 1 : 0;
    if (timer.on) ck(gls_section_timing(ctx, 1), "gls_section_timing");
    ck(gls_newton_solve(ctx, d_present, d_m1, d_m2, d_m3, &np), "gls_newton_solve");
    if (timer.on) {  // the library's Newton / GMRES sections (gls_navier_stokes.cc:921, 1028, 1165, 1274)
      static const char *names[GLS_N_SECTIONS] = {"assemble_system", "assemble_rhs", "setup_ILU", "setup_GMG",
                                                  "solve_linear_system"};
      for (int sct = 0; sct < GLS_N_SECTIONS; ++sct) {
        double sec = 0;
        int calls = 0;
        ck(gls_section_get(ctx, sct, &sec, &calls), "gls_section_get");
        if (calls > 0) timer.add(names[sct], calls, sec);
      }
      ck(gls_section_timing(ctx, 0), "gls_section_timing");
    }
    if (np.linear_failures > 0)
      printf("  -Warning: %d linear solve(s) stopped at the iteration limit before the tolerance\n", np.linear_failures);
    dev_changed();
    newton_its += np.newton_iterations;
    linear_its += np.linear_iterations;
    if (nu_override > 0) ck(gls_set_viscosity(ctx, P.nu), "gls_set_viscosity");
  }
  void push_dt(double dt) {  // the newest step first, older ones shifted
    for (int i = 3; i > 0; --i) dts[i] = dts[i - 1];
    dts[0] = dt;
    dt_now = dt;
  }

  // one time step with the scheme's stages (SDIRK stage results become m2 / m3)
  void advance() {
    if (P.method == Method::sdirk2) {
      solve_nonlinear(GLS_SDIRK2_1);
      dcopy(d_m2, d_present);
      solve_nonlinear(GLS_SDIRK2_2);
    } else if (P.method == Method::sdirk3) {
      solve_nonlinear(GLS_SDIRK3_1);
      dcopy(d_m2, d_present);
      solve_nonlinear(GLS_SDIRK3_2);
      dcopy(d_m3, d_present);
      solve_nonlinear(GLS_SDIRK3_3);
    } else {
      const int sch[] = {GLS_STEADY, GLS_BDF1, GLS_BDF2, GLS_BDF3};
      solve_nonlinear(sch[(int)P.method]);
    }
  }
  // first step of BDF2 / BDF3: Euler sub-steps of `startup`*dt, then the high-order step
  // completing dt (navier_stokes_base.cc:507-586)
  void first_step() {
    if (P.method != Method::bdf2 && P.method != Method::bdf3) {
      advance();
      return;
    }
    const double dt = P.dt, s = P.startup;
    push_dt(dt * s);
    solve_nonlinear(GLS_BDF1, -1.0, true);  // start-up solves force a fresh matrix (:534-574)
    dcopy(d_m2, d_m1);
    dcopy(d_m1, d_present);
    if (P.method == Method::bdf2) {
      push_dt(dt * (1. - s));
      solve_nonlinear(GLS_BDF2, -1.0, true);
    } else {
      push_dt(dt * s);
      solve_nonlinear(GLS_BDF1, -1.0, true);
      dcopy(d_m3, d_m2);
      dcopy(d_m2, d_m1);
      dcopy(d_m1, d_present);
      push_dt(dt * (1. - 2. * s));
      solve_nonlinear(GLS_BDF3, -1.0, true);
    }
    dt_now = dt;
  }

  // ---- post-processing
  std::pair<double, double> l2_error() {  // QGauss(k+2), pressures compared mean-free
    SectionTimer::Scope ts(timer, "error");
    CellEval ev(m, m.k + 2);
    std::vector<double> X, E;
    for (int64_t c = 0; c < m.nc; ++c)
      for (int q = 0; q < ev.nq; ++q) {
        double x[3], w;
        ev.point(c, q, x, w);
        X.insert(X.end(), x, x + m.dim);
      }
    P.exact.eval(X, m.dim, time, E);
    const int ne = P.exact.nc;
    double pint = 0, peint = 0, vol = 0, eu = 0, ep = 0;
    // GridTools::volume(triangulation) = the Q1 measure of the cells (navier_stokes_base.cc:320)
    if (m.general)
      for (double v : m.measure) vol += v;
    for (int pass = 0; pass < 2; ++pass) {
      int64_t idx = 0;
      for (int64_t c = 0; c < m.nc; ++c)
        for (int q = 0; q < ev.nq; ++q, ++idx) {
          double x[3], JxW, u[3], G[3][3], p;
          ev.point(c, q, x, JxW);
          ev.at(present.data(), c, q, u, G, p);
          const double *ex = &E[(size_t)(idx * ne)];
          const double pe = ne > m.dim ? ex[m.dim] : 0.0;
          if (pass == 0) {
            pint += p * JxW;
            peint += pe * JxW;
            vol += m.general ? 0.0 : JxW;
          } else {
            for (int d = 0; d < m.dim; ++d) eu += (u[d] - ex[d]) * (u[d] - ex[d]) * JxW;
            const double dp = (p - pint / vol) - (pe - peint / vol);
            ep += dp * dp * JxW;
          }
        }
    }
    return {std::sqrt(eu), std::sqrt(ep)};
  }
  // volume averages with QGauss(k+1): 0.5|curl u|^2 (enstrophy) or 0.5|u|^2 (kinetic energy)
  double volume_average(bool enstrophy) {
    CellEval ev(m, std::max(m.k, m.kp) + 1);
    double s = 0, vol = 0;
    for (int64_t c = 0; c < m.nc; ++c)
      for (int q = 0; q < ev.nq; ++q) {
        double x[3], JxW, u[3], G[3][3], p;
        ev.point(c, q, x, JxW);
        ev.at(present.data(), c, q, u, G, p);
        vol += JxW;
        if (enstrophy) {
          const double wz = G[1][0] - G[0][1];
          s += 0.5 * wz * wz * JxW;
          if (m.dim == 3) {
            const double wx = G[2][1] - G[1][2], wy = G[0][2] - G[2][0];
            s += 0.5 * (wx * wx + wy * wy) * JxW;
          }
        } else {
          for (int d = 0; d < m.dim; ++d) s += 0.5 * u[d] * u[d] * JxW;
        }
      }
    return s / vol;
  }
  // CFL from the velocity at the cell centre and h = (6|K|/pi)^(1/3)/k (3D), sqrt(4|K|/pi)/k (2D)
  double compute_cfl(double dt) {
    if (!m.general && m.vx.empty() && m.k <= 2) {  // box cells: on the device, from d_present
      const int k1 = m.k + 1, nvl = m.dim == 3 ? k1 * k1 * k1 : k1 * k1;
      const int64_t nb = (m.nc + 255) / 256;
      if (!d_cv) {
        hk(hipMalloc(&d_cv, sizeof(int32_t) * m.cv.size()), "hipMalloc");
        hk(hipMalloc(&d_h, sizeof(double) * m.h.size()), "hipMalloc");
        hk(hipMalloc(&d_blk, sizeof(double) * (size_t)nb), "hipMalloc");
        hk(hipMemcpy(d_cv, m.cv.data(), sizeof(int32_t) * m.cv.size(), hipMemcpyHostToDevice), "upload");
        hk(hipMemcpy(d_h, m.h.data(), sizeof(double) * m.h.size(), hipMemcpyHostToDevice), "upload");
      }
      need_dev();
      double b[3] = {0, 0, 0}, db[4];
      lag1d(lobatto01(m.k), 0.5, b, db);
      hk(hipDeviceSynchronize(), "cfl");
      hipLaunchKernelGGL(k_cfl, dim3((unsigned)nb), dim3(256), 0, 0, d_cv, d_h, d_present, m.nc, m.dim, nvl, k1, b[0], b[1],
                         b[2], (double)std::max(m.k, m.kp), dt, d_blk);
      hk(hipGetLastError(), "k_cfl");
      std::vector<double> bm((size_t)nb);
      hk(hipMemcpy(bm.data(), d_blk, sizeof(double) * (size_t)nb, hipMemcpyDeviceToHost), "download");
      return *std::max_element(bm.begin(), bm.end());
    }
    need_host();
    CellEval ev(m, 1);
    const int deg = std::max(m.k, m.kp);
    double cmax = 0;
    for (int64_t c = 0; c < m.nc; ++c) {
      double u[3], G[3][3], p, meas = 1;
      ev.at(present.data(), c, 0, u, G, p);
      if (m.general) meas = m.measure[(size_t)c];
      else
        for (int d = 0; d < m.dim; ++d) meas *= m.h[(size_t)(c * m.dim + d)];
      const double hh = m.dim == 2 ? std::sqrt(4. * meas / M_PI) / deg : std::cbrt(6. * meas / M_PI) / deg;
      double un = 0;
      for (int d = 0; d < m.dim; ++d) un += u[d] * u[d];
      cmax = std::max(cmax, std::sqrt(un) / hh * dt);
    }
    return cmax;
  }
  void write_output() {
    SectionTimer::Scope ts(timer, "output");
    need_host();
    if (rank != 0) return;  // --np: rank 0 writes the (gathered) solution
    char tag[32];
    std::snprintf(tag, sizeof(tag), ".%05d", step);
    const std::string stem = P.output_name + tag, piece = stem + ".00000.vtu", master = stem + ".pvtu";
    gls_mesh_desc D;
    std::memset(&D, 0, sizeof(D));
    D.dim = m.dim;
    D.k = m.k;
    D.kp = m.kp;
    D.n_cells = (int)m.nc;
    D.n_vnodes = (int)m.nv;
    D.n_pnodes = (int)m.np;
    D.cell_vnodes = m.cv.data();
    D.cell_pnodes = m.cp.data();
    if (m.general) {
      D.map_degree = m.k;
      D.cell_support = m.support.data();
    } else {
      D.cell_x0 = m.x0.data();
      D.cell_h = m.h.data();
    }
    D.srf = P.srf ? 1 : 0;
    for (int i = 0; i < 3; ++i) D.omega[i] = P.omega[i];
    ck(gls_vtu_write((P.output_path + piece).c_str(), &D, present.data(), P.subdivision, 0, 1), "gls_vtu_write");
    const char *pc[1] = {piece.c_str()};
    ck(gls_pvtu_write((P.output_path + master).c_str(), m.dim, P.srf ? 1 : 0, 1, pc), "gls_pvtu_write");
    pvd.emplace_back(time, master);
    std::vector<double> tt;
    std::vector<const char *> ff;
    for (auto &e : pvd) {
      tt.push_back(e.first);
      ff.push_back(e.second.c_str());
    }
    ck(gls_pvd_write((P.output_path + P.output_name + ".pvd").c_str(), (int)pvd.size(), tt.data(), ff.data()),
       "gls_pvd_write");
  }
  void postprocess(bool initial) {
    if (P.output_frequency > 0 && step % P.output_frequency == 0) write_output();
    if (P.enstrophy || P.kinetic || (!initial && P.analytical)) need_host();
    // post-processing lines of NavierStokesBase::postprocess (navier_stokes_base.cc:791-853)
    if (P.enstrophy && P.pp_verbose) std::printf("Enstrophy  : %s\n", g6(volume_average(true)).c_str());
    if (P.kinetic) {  // navier_stokes_base.cc:824-839
      SectionTimer::Scope ts(timer, "kinetic_energy_calculation");
      const double ke = volume_average(false);
      if (P.pp_verbose) std::printf("Kinetic energy : %s\n", g6(ke).c_str());
    }
    if (!initial && P.analytical) {
      const auto e = l2_error();
      if (P.method == Method::steady) errors.push_back({(double)m.nc, e.first, e.second});
      else errors.push_back({time, e.first});
      if (P.analytical_verbose && P.method != Method::steady)
        std::printf("L2 error velocity : %s\n", g6(e.first).c_str());
    }
  }
  void end_of_step() {  // history shift (device: pointer rotation + one copy) + CFL of the step just taken
    if (P.method == Method::steady) return;
    need_dev();
    double *t = d_m3;
    d_m3 = d_m2;
    d_m2 = d_m1;
    d_m1 = t;
    dcopy(d_m1, d_present);
    dev_changed();
    cfl = compute_cfl(dt_now);
  }
  // uniform refinement with interpolation of the Qk fields onto the refined lattice
  void refine_uniform() {
    SectionTimer::Scope ts(timer, "refine");
    need_host();
    if (m.general) {  // refine_global + SolutionTransfer (gls_fe_space_transfer)
      const std::vector<double> sol = present;
      gls_fe_space *old_space = space;
      space = nullptr;  // keep the old space alive across setup_general
      ck(gls_umesh_refine_global(um, 1), "refine_global");
      setup_general();
      ck(gls_fe_space_transfer(old_space, space, sol.data(), present.data()), "gls_fe_space_transfer");
      gls_fe_space_destroy(old_space);
      host_changed();
      return;
    }
    const Mesh old = m;
    const std::vector<double> sol = present;
    setup(m.n * 2);
    const int dim = old.dim;
    auto value_at = [&](const double *x, int comp) {
      const bool vel = comp < dim;
      const int kk = (vel ? old.k : old.kp) + 1;
      const std::vector<double> xn = lobatto01(kk - 1);
      int ci[3] = {0, 0, 0};
      double b[3][4], db[4];
      for (int d = 0; d < dim; ++d) {
        const double s = (x[d] - old.lo) / old.hc;
        ci[d] = std::min((int)std::floor(s), old.n - 1);
        lag1d(xn, s - ci[d], b[d], db);
      }
      const int nl = dim == 3 ? kk * kk * kk : kk * kk;
      double s = 0;
      for (int a = 0; a < nl; ++a) {
        const int la[3] = {a % kk, (a / kk) % kk, dim == 3 ? a / (kk * kk) : 0};
        int64_t id = 0, stride = 1;
        for (int d = 0; d < dim; ++d) {
          const int sh = vel ? old.vsh[d] : old.psh[d];
          id += (int64_t)((ci[d] * (kk - 1) + la[d]) % sh) * stride;
          stride *= sh;
        }
        const double w = b[0][la[0]] * b[1][la[1]] * (dim == 3 ? b[2][la[2]] : 1.0);
        s += w * (vel ? sol[(size_t)(id * dim + comp)] : sol[(size_t)(dim * old.nv + id)]);
      }
      return s;
    };
    for (int part = 0; part < 2; ++part) {
      const bool vel = part == 0;
      for (int64_t v = 0; v < (vel ? m.nv : m.np); ++v) {
        double x[3];
        int idx[3];
        m.coord(v, vel, x, idx);
        if (vel)
          for (int d = 0; d < dim; ++d) present[(size_t)(v * dim + d)] = value_at(x, d);
        else
          present[(size_t)(dim * m.nv + v)] = value_at(x, dim);
      }
    }
    host_changed();
  }
  // refine_mesh_kelly (navier_stokes_base.cc:610-780): Kelly indicator of the velocity or pressure
  // on the device (gls_kelly_estimate on the uniform mesh, gls_kelly_estimate_faces on an adapted
  // one; stored as float like deal.II's Vector<float>), refine_and_coarsen_fixed_{number,fraction}
  // with coarsening (:654-667), the max / min refinement level rules (:669-680),
  // prepare_coarsening_and_refinement with the triangulation's smoothing (:682), execution on the
  // forest (refine, coarsen complete families, corner balance: p4est) and SolutionTransfer of the
  // present solution (:684-733). The forest is the hyper_cube's one coarse cell refined
  // `initial refinement` times, so leaf levels are deal.II's cell levels.
  void refine_kelly() {
    SectionTimer::Scope ts(timer, "refine");
    if (m.general) {
      refine_kelly_general();
      return;
    }
    need_host();
    const int dim = P.dim;
    const int64_t nc = m.nc;
    upload(present, d_present);
    double *d_eta = nullptr;
    hk(hipMalloc(&d_eta, sizeof(double) * (size_t)nc), "hipMalloc");
    if (!rmesh) {
      ck(gls_kelly_estimate(ctx, d_present, P.kelly_variable, d_eta), "gls_kelly_estimate");
    } else {
      int64_t nf = 0;
      ck(gls_octree_faces(rmesh, &nf, nullptr, nullptr, nullptr, nullptr, nullptr), "gls_octree_faces");
      std::vector<int32_t> fa((size_t)nf), fb((size_t)nf), fd((size_t)nf);
      std::vector<double> ra((size_t)nf * 4), rb((size_t)nf * 4);
      ck(gls_octree_faces(rmesh, &nf, fa.data(), fb.data(), fd.data(), ra.data(), rb.data()), "gls_octree_faces");
      ck(gls_kelly_estimate_faces(ctx, d_present, P.kelly_variable, nf, fa.data(), fb.data(), fd.data(), ra.data(),
                                  rb.data(), d_eta),
         "gls_kelly_estimate_faces");
    }
    hk(hipDeviceSynchronize(), "kelly estimate");  // the context stream is not the null stream
    std::vector<double> eta((size_t)nc);
    download(d_eta, eta);
    (void)hipFree(d_eta);
    const int64_t n_uniform = (int64_t)1 << P.refinement;
    gls_refined_mesh *um = nullptr;  // periodic: the uniform mesh as the forest numbers it (SolutionTransfer source)
    if (!tree) {  // GridGenerator::hyper_cube + refine_global(initial refinement)
      if (rmesh) die("kelly mesh adaptation: internal error (adapted mesh without a forest)");
      ck(gls_octree_create(dim, 1, &tree), "gls_octree_create");
      ck(gls_octree_set_periodic(tree, m.pmask), "gls_octree_set_periodic");  // add_periodicity
      for (int r = 0; r < P.refinement; ++r) {
        int64_t nl = 0;
        ck(gls_octree_info(tree, &nl, nullptr), "gls_octree_info");
        std::vector<int32_t> all((size_t)nl, 1), none((size_t)nl, 0);
        ck(gls_octree_adapt(tree, all.data(), none.data(), 1 << 20, 0), "gls_octree_adapt");
      }
      if (m.pmask) {  // the wrapped uniform lattice in lexicographic order is the forest mesh's numbering
        ck(gls_octree_mesh(tree, P.k, P.kp, P.lo, P.hi, &um), "gls_octree_mesh");
        bool same = um->n_vnodes == m.nv && um->n_pnodes == m.np;
        for (int64_t v = 0; same && v < m.nv; ++v) {
          double x[3];
          int idx[3];
          m.coord(v, true, x, idx);
          for (int d = 0; d < dim; ++d) same = same && std::fabs(x[d] - um->vnode_x[v * dim + d]) < 1e-12 * (P.hi - P.lo);
        }
        if (!same) die("kelly mesh adaptation: periodic uniform mesh and forest numbering disagree");
      }
    }
    int64_t nl = 0;
    int max_lev = 0;
    ck(gls_octree_info(tree, &nl, &max_lev), "gls_octree_info");
    if (nl != nc) die("kelly mesh adaptation: forest (%lld leaves) and mesh (%lld cells) disagree", (long long)nl, (long long)nc);
    std::vector<int32_t> lev((size_t)nl);
    std::vector<double> x0((size_t)nl * dim), hh((size_t)nl * dim);
    ck(gls_octree_cells(tree, lev.data(), x0.data(), hh.data(), P.lo, P.hi), "gls_octree_cells");
    std::vector<float> crit((size_t)nc);
    if (!rmesh) {  // the uniform mesh's cell order -> the forest's leaf order
      const double hc = (P.hi - P.lo) / (double)n_uniform;
      std::vector<int64_t> at((size_t)nc);
      for (int64_t c = 0; c < nc; ++c) {
        int64_t lex = 0, st = 1;
        for (int d = 0; d < dim; ++d) {
          lex += std::lround((m.x0[(size_t)(c * dim + d)] - P.lo) / hc) * st;
          st *= n_uniform;
        }
        at[(size_t)lex] = c;
      }
      for (int64_t i = 0; i < nl; ++i) {
        int64_t lex = 0, st = 1;
        for (int d = 0; d < dim; ++d) {
          lex += std::lround((x0[(size_t)(i * dim + d)] - P.lo) / hc) * st;
          st *= n_uniform;
        }
        crit[(size_t)i] = (float)eta[(size_t)at[(size_t)lex]];
      }
    } else {
      for (int64_t i = 0; i < nc; ++i) crit[(size_t)i] = (float)eta[(size_t)i];
    }
    std::vector<int32_t> rf((size_t)nc, 0), cf((size_t)nc, 0);
    ck(gls_refine_coarsen_pd(nc, crit.data(), dim, P.frac_type, P.frac_refine, P.frac_coarsen, P.max_cells,
                             rf.data(), cf.data(), nullptr),
       "gls_refine_coarsen_pd");
    int64_t nr0 = 0, nc0 = 0;
    for (int64_t i = 0; i < nc; ++i) {
      nr0 += rf[(size_t)i];
      nc0 += cf[(size_t)i];
    }
    // tria.n_levels() > max refinement level: no refinement from that level up; no coarsening on
    // the min refinement level
    for (int64_t i = 0; i < nc; ++i) {
      if (max_lev + 1 > P.max_level && lev[(size_t)i] >= P.max_level) rf[(size_t)i] = 0;
      if (lev[(size_t)i] == P.min_level) cf[(size_t)i] = 0;
    }
    ck(gls_octree_prepare(tree, rf.data(), cf.data()), "gls_octree_prepare");
    int64_t nr1 = 0, nc1 = 0;
    for (int64_t i = 0; i < nc; ++i) {
      nr1 += rf[(size_t)i];
      nc1 += cf[(size_t)i];
    }
    std::printf("kelly: %lld of %lld cells flagged for refinement, %lld for coarsening (after smoothing: %lld, %lld)\n",
                (long long)nr0, (long long)nc, (long long)nc0, (long long)nr1, (long long)nc1);
    ck(gls_octree_adapt(tree, rf.data(), cf.data(), 1 << 20, 0), "gls_octree_adapt");
    gls_refined_mesh *nm = nullptr;
    ck(gls_octree_mesh(tree, P.k, P.kp, P.lo, P.hi, &nm), "gls_octree_mesh");
    // SolutionTransfer of the present solution and, transient, the time history (:684-733)
    const bool transient = P.method != Method::steady;
    const std::vector<double> sol = present, s1 = m1, s2 = m2, s3 = m3;
    gls_refined_mesh *old_rm = rmesh;
    rmesh = nullptr;  // kept for the transfer (release() would free it)
    setup_refined(nm);
    host_changed();  // present (and the history) are rewritten on the host below
    auto move = [&](const std::vector<double> &from, std::vector<double> &to) {
      if (old_rm) ck(gls_octree_transfer(old_rm, rmesh, from.data(), to.data()), "gls_octree_transfer");
      else if (um) ck(gls_octree_transfer(um, rmesh, from.data(), to.data()), "gls_octree_transfer");
      else ck(gls_mesh_refined_interpolate(rmesh, (int)n_uniform, P.lo, P.hi, from.data(), to.data()),
              "gls_mesh_refined_interpolate");
    };
    move(sol, present);
    if (transient) {
      move(s1, m1);
      move(s2, m2);
      move(s3, m3);
    }
    if (old_rm) gls_octree_mesh_destroy(old_rm);
    if (um) gls_octree_mesh_destroy(um);
  }
  // refine_mesh_kelly on a general (gmsh / GridGenerator, curved) triangulation: the Kelly indicator
  // with MappingQ face geometry (gls_fe_space_kelly_faces + gls_kelly_estimate_mapped), the same
  // thresholds and level rules as above, prepare_coarsening_and_refinement / execution on the
  // triangulation's hierarchy (gls_umesh_prepare / gls_umesh_adapt), SolutionTransfer of the present
  // solution and the time history (navier_stokes_base.cc:684-780)
  void refine_kelly_general() {
    need_host();
    const int dim = P.dim;
    const int64_t nc = m.nc;
    const int nq = P.k + 2;  // QGauss<dim-1>(n_q + 1), n_q = velocity order + 1
    const int nqf = dim == 3 ? nq * nq : nq;
    int64_t np = 0;
    ck(gls_fe_space_kelly_faces(space, nq, &np, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr), "gls_fe_space_kelly_faces");
    std::vector<int32_t> ca((size_t)np), cb((size_t)np);
    std::vector<double> xi((size_t)(np * nqf * 2 * dim)), g(xi.size()), jxw((size_t)(np * nqf)), diam((size_t)nc);
    ck(gls_fe_space_kelly_faces(space, nq, &np, ca.data(), cb.data(), xi.data(), g.data(), jxw.data(), diam.data()),
       "gls_fe_space_kelly_faces");
    std::vector<double> eta((size_t)nc);
    if (world == 1 || rank == 0) {  // --np: rank 0 on a context of the whole mesh, eta broadcast
      gls_ctx *kc = world > 1 ? make_context(m, C) : ctx;
      double *d_eta = nullptr, *d_sol = d_present;
      hk(hipMalloc(&d_eta, sizeof(double) * (size_t)std::max<int64_t>(nc, 1)), "hipMalloc");
      if (world > 1) hk(hipMalloc(&d_sol, sizeof(double) * present.size()), "hipMalloc");
      hk(hipMemcpy(d_sol, present.data(), sizeof(double) * present.size(), hipMemcpyHostToDevice), "upload");
      ck(gls_kelly_estimate_mapped(kc, d_sol, P.kelly_variable, np, nqf, ca.data(), cb.data(), xi.data(), g.data(),
                                   jxw.data(), diam.data(), d_eta),
         "gls_kelly_estimate_mapped");
      hk(hipDeviceSynchronize(), "kelly estimate");
      hk(hipMemcpy(eta.data(), d_eta, sizeof(double) * eta.size(), hipMemcpyDeviceToHost), "download");
      (void)hipFree(d_eta);
      if (world > 1) {
        (void)hipFree(d_sol);
        gls_destroy(kc);
      }
    }
    if (world > 1) g_comm.bcast(eta, 0);
    std::vector<float> crit((size_t)nc);
    int max_lev = 0;
    for (int64_t i = 0; i < nc; ++i) {
      crit[(size_t)i] = (float)eta[(size_t)i];
      max_lev = std::max(max_lev, (int)space->cell_level[i]);
    }
    std::vector<int32_t> rf((size_t)nc, 0), cf((size_t)nc, 0);
    ck(gls_refine_coarsen_pd(nc, crit.data(), dim, P.frac_type, P.frac_refine, P.frac_coarsen, P.max_cells, rf.data(),
                             cf.data(), nullptr),
       "gls_refine_coarsen_pd");
    int64_t nr0 = 0, nc0 = 0;
    for (int64_t i = 0; i < nc; ++i) {
      nr0 += rf[(size_t)i];
      nc0 += cf[(size_t)i];
    }
    for (int64_t i = 0; i < nc; ++i) {  // max / min refinement level rules (:669-680)
      if (max_lev + 1 > P.max_level && space->cell_level[i] >= P.max_level) rf[(size_t)i] = 0;
      if (space->cell_level[i] == P.min_level) cf[(size_t)i] = 0;
    }
    ck(gls_umesh_prepare(um, rf.data(), cf.data()), "gls_umesh_prepare");
    int64_t nr1 = 0, nc1 = 0;
    for (int64_t i = 0; i < nc; ++i) {
      nr1 += rf[(size_t)i];
      nc1 += cf[(size_t)i];
    }
    if (stats)
      std::printf("kelly: %lld of %lld cells flagged for refinement, %lld for coarsening (after smoothing: %lld, %lld)\n",
                  (long long)nr0, (long long)nc, (long long)nc0, (long long)nr1, (long long)nc1);
    ck(gls_umesh_adapt(um, rf.data(), cf.data()), "gls_umesh_adapt");
    const std::vector<double> s0 = present, s1 = m1, s2 = m2, s3 = m3;
    gls_fe_space *old_space = space;
    space = nullptr;  // keep the old space alive across setup_general
    setup_general();
    ck(gls_fe_space_transfer(old_space, space, s0.data(), present.data()), "gls_fe_space_transfer");
    if (P.method != Method::steady) {
      ck(gls_fe_space_transfer(old_space, space, s1.data(), m1.data()), "gls_fe_space_transfer");
      ck(gls_fe_space_transfer(old_space, space, s2.data(), m2.data()), "gls_fe_space_transfer");
      ck(gls_fe_space_transfer(old_space, space, s3.data(), m3.data()), "gls_fe_space_transfer");
    }
    gls_fe_space_destroy(old_space);
    host_changed();
  }
  // NavierStokesBase::finish_simulation's error table (navier_stokes_base.cc:382-424): deal.II
  // ConvergenceTable text layout — steady: cells | error_velocity + log2 reduction rate |
  // error_pressure + rate, errors in scientific notation with `precision` digits, rates fixed 2,
  // "-" where no rate, supercolumn headers centred over their span; transient: time (fixed 4) |
  // error_velocity
  void report() {
    if (!P.analytical || errors.empty()) return;
    std::ostringstream o;
    auto sci = [&](double v) {
      char b[64];
      std::snprintf(b, sizeof(b), "%.*e", precision, v);
      return std::string(b);
    };
    auto fixed = [](double v, int d) {
      char b[64];
      std::snprintf(b, sizeof(b), "%.*f", d, v);
      return std::string(b);
    };
    auto rpad = [](const std::string &t, size_t w) { return std::string(w > t.size() ? w - t.size() : 0, ' ') + t; };
    auto lpad = [](const std::string &t, size_t w) { return t + std::string(w > t.size() ? w - t.size() : 0, ' '); };
    auto centre = [](const std::string &t, size_t w) {
      const size_t f = w > t.size() ? (w - t.size()) / 2 : 0, r = w > t.size() ? w - t.size() - f : 0;
      return std::string(f, ' ') + t + std::string(r, ' ');
    };
    const size_t n = errors.size();
    if (P.method == Method::steady) {
      std::vector<std::string> c0, eu, ru, ep, rp;
      for (size_t i = 0; i < n; ++i) {
        const auto &r = errors[i];
        c0.push_back(std::to_string((long long)r[0]));
        eu.push_back(sci(r[1]));
        ep.push_back(sci(r[2]));
        ru.push_back(i ? fixed(std::log2(errors[i - 1][1] / r[1]), 2) : "-");
        rp.push_back(i ? fixed(std::log2(errors[i - 1][2] / r[2]), 2) : "-");
      }
      auto width = [](const std::vector<std::string> &v, size_t w0) {
        size_t w = w0;
        for (auto &t : v) w = std::max(w, t.size());
        return w;
      };
      const size_t w0 = width(c0, 5), w1 = width(eu, 0), w2 = width(ru, 0), w3 = width(ep, 0), w4 = width(rp, 0);
      o << centre("cells", w0) << ' ' << centre("error_velocity", w1 + 1 + w2) << ' '
        << centre("error_pressure", w3 + 1 + w4) << ' ' << '\n';
      for (size_t i = 0; i < n; ++i)
        o << rpad(c0[i], w0) << ' ' << rpad(eu[i], w1) << ' ' << rpad(ru[i], w2) << ' ' << rpad(ep[i], w3) << ' '
          << rpad(rp[i], w4) << ' ' << '\n';
    } else {
      std::vector<std::string> t0, eu;
      for (auto &r : errors) {
        t0.push_back(fixed(r[0], 4));
        eu.push_back(sci(r[1]));
      }
      size_t w0 = 4, w1 = 14;
      for (auto &t : t0) w0 = std::max(w0, t.size());
      for (auto &t : eu) w1 = std::max(w1, t.size());
      o << centre("time", w0) << ' ' << centre("error_velocity", w1) << ' ' << '\n';
      for (size_t i = 0; i < n; ++i) o << rpad(t0[i], w0) << ' ' << lpad(eu[i], w1) << ' ' << '\n';
    }
    std::printf("%s", o.str().c_str());
    std::ofstream(P.analytical_file + ".dat") << o.str();
  }

  void run() {
    dt_now = P.dt;
    dts[0] = P.dt;
    std::printf("Running on %d MPI rank(s)...\n", world);  // navier_stokes_base.cc:115-117 (one rank per GPU)
    if (world > 1 && !P.general) P.general = true;  // --np: every mesh through the general (partitioned) path
    if (P.general) {
      create_umesh();
      setup_general();
    } else {
      setup(1 << P.refinement);
    }
    if (P.ic_type == "nodal" || P.ic_type == "viscous") {
      nodal_values(P.ic, present);
      host_changed();
      if (P.ic_type == "viscous") solve_nonlinear(GLS_STEADY, P.ic_nu);
    } else if (P.ic_type == "L2projection") {
      l2_projection(P.ic, present);
      host_changed();
    } else {
      die("initial condition type '%s' is not supported", P.ic_type.c_str());
    }
    end_of_step();
    postprocess(true);
    const bool steady = P.method == Method::steady;
    while (steady ? step < P.mesh_adapt + 1 : time < P.t_end - 1e-12 * dt_now) {
      ++step;
      if (steady) {
        time = step;
      } else {
        const double dt = std::min(dt_now, P.t_end - time);
        push_dt(dt);
        time += dt;
      }
      if (P.log_frequency > 0 && step % P.log_frequency == 0) {
        // SimulationControl{Steady,Transient}::print_progression (simulation_control.cc:92-107, 242-255)
        const char *stars = "*****************************************************************";
        if (steady)
          std::printf("\n%s\nSteady iteration : %8d/%d\n%s\n", stars, step, P.mesh_adapt + 1, stars);
        else
          std::printf("\n%s\nTransient iteration : %-8d Time : %-8s Time step : %-8s CFL : %-8s\n%s\n", stars, step,
                      g6(time).c_str(), g6(dt_now).c_str(), g6(cfl).c_str(), stars);
      }
      if (step == 1) {
        first_step();
      } else {
        if (step % P.adapt_frequency == 0) {  // refine_mesh (navier_stokes_base.cc:592-607)
          if (P.madapt == "kelly") refine_kelly();  // steady and transient (gls_navier_stokes.cc:1406-1416)
          else if (steady) refine_uniform();
        }
        advance();
      }
      postprocess(false);
      dump_state();
      end_of_step();
      if (P.timer == "iteration") {  // TimerOutput print_summary + reset per iteration (navier_stokes_base.cc:449-455)
        timer.print();
        timer.reset();
      }
    }
    report();
    timer.print();  // the TimerOutput destructor's summary (output frequency 'summary')
    if (stats) std::printf("newton_iterations = %d, linear_iterations = %d\n", newton_its, linear_its);
  }
};

}  // namespace

int main(int argc, char **argv) {
  // gls_navier_stokes_2d / gls_navier_stokes_3d <file.prm> (applications/gls_navier_stokes_{2d,3d},
  // gls_navier_stokes_3d.cc:22-46): the dimension comes from the program name; the generic
  // binary takes --dim. Extra options: --precond mg|ilu|hmg|jacobi (ilu: never the refinement-hierarchy
  // multigrid on adapted meshes; hmg: that multigrid for every method and order), --precision N (error table digits),
  // --stats (solver iteration totals), --ilu-block-dofs N (block-Jacobi ILU subdomains of N DoFs,
  // 0 = one block), --ilu-order cm|multicolor (gls_ilu_set_options), --dump DIR (every iteration's
  // final state for the pipeline tests).
  int dim = 0;
  bool mg = true, stats = false;
  int64_t ilu_block = -1;
  int ilu_order = -1;
  const char *dump = nullptr;
  int np_ranks = 1;
  int forest_mode = 0;
  int precision = 4;
  const char *file = nullptr;
  const std::string prog = argv[0];
  if (prog.size() >= 2 && prog.compare(prog.size() - 2, 2, "2d") == 0) dim = 2;
  if (prog.size() >= 2 && prog.compare(prog.size() - 2, 2, "3d") == 0) dim = 3;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--dim") && i + 1 < argc) dim = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--precond") && i + 1 < argc) {
      const char *pc = argv[++i];
      if (std::strcmp(pc, "mg") && std::strcmp(pc, "jacobi") && std::strcmp(pc, "ilu") && std::strcmp(pc, "hmg"))
        die("--precond %s: mg, ilu, hmg or jacobi", pc);
      mg = std::strcmp(pc, "jacobi") != 0;
      forest_mode = !std::strcmp(pc, "ilu") ? 1 : !std::strcmp(pc, "hmg") ? 2 : 0;
    }
    else if (!std::strcmp(argv[i], "--precision") && i + 1 < argc) precision = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--stats")) stats = true;
    else if (!std::strcmp(argv[i], "--ilu-block-dofs") && i + 1 < argc) ilu_block = std::atoll(argv[++i]);
    else if (!std::strcmp(argv[i], "--dump") && i + 1 < argc) dump = argv[++i];
    else if (!std::strcmp(argv[i], "--np") && i + 1 < argc) np_ranks = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--ilu-order") && i + 1 < argc) {
      const char *o = argv[++i];
      if (!std::strcmp(o, "cm")) ilu_order = GLS_ILU_ORDER_CM;
      else if (!std::strcmp(o, "multicolor")) ilu_order = GLS_ILU_ORDER_MULTICOLOR;
      else die("--ilu-order %s: cm or multicolor", o);
    }
    else if (argv[i][0] != '-') file = argv[i];
    else die("unknown option %s", argv[i]);
  }
  if (!file) {  // the reference prints its usage and exits 1 (gls_navier_stokes_3d.cc:27-31)
    std::printf("Usage:\n%s input_file\n", argv[0]);
    return 1;
  }
  if (dim == 0) dim = 3;
  if (dim != 2 && dim != 3) die("--dim must be 2 or 3");
  std::setvbuf(stdout, nullptr, _IOLBF, 0);  // progress visible in a log while the run goes on
  Prm prm(file);
  Params P = read_params(prm, dim);
  // --np N: N ranks forked here, before any GPU call (the children's stdout is discarded: rank 0
  // prints, as the reference's pcout does)
  if (np_ranks < 1 || np_ranks > kMaxRanks) die("--np must be in 1..%d", kMaxRanks);
  int rank = 0;
  std::vector<pid_t> kids;
  if (np_ranks > 1) {
    g_comm.create(np_ranks);
    std::fflush(stdout);
    std::fflush(stderr);
    for (int r = 1; r < np_ranks; ++r) {
      const pid_t pid = fork();
      if (pid < 0) die("--np: fork failed");
      if (pid == 0) {
        rank = r;
        kids.clear();
        if (!std::freopen("/dev/null", "w", stdout)) die("--np: /dev/null");
        break;
      }
      kids.push_back(pid);
    }
    g_comm.rank = rank;
  }
  Solver s(P, mg);
  s.forest_mode = forest_mode;
  s.rank = rank;
  s.world = np_ranks;
  if (np_ranks > 1) {
    int ndev = 0;
    hk(hipGetDeviceCount(&ndev), "hipGetDeviceCount");
    hk(hipSetDevice(rank % std::max(ndev, 1)), "hipSetDevice");
    if (ndev >= np_ranks && !std::getenv("GLS_NP_SHM")) {  // one GPU per rank: RCCL over xGMI
      if (rank == 0) ck(gls_rccl_unique_id(g_comm.hdr->rccl_id), "gls_rccl_unique_id");
      g_comm.barrier("rccl-id");
      ck(gls_rccl_create(g_comm.hdr->rccl_id, rank, np_ranks, &s.rccl), "gls_rccl_create");
    }
  }
  s.precision = precision;
  s.stats = stats;
  if (ilu_block >= 0) s.ilu_block_dofs = ilu_block;
  s.ilu_order = ilu_order;
  if (dump) s.dump_dir = dump;
  s.run();
  if (np_ranks > 1) {
    g_comm.barrier("end");
    s.release();
    if (s.rccl) gls_rccl_destroy(s.rccl);
    if (rank != 0) {
      std::fflush(stderr);
      _exit(0);
    }
    int bad = 0;
    for (pid_t pid : kids) {
      int st = 0;
      if (waitpid(pid, &st, 0) < 0 || !WIFEXITED(st) || WEXITSTATUS(st) != 0) ++bad;
    }
    if (bad) die("--np: %d rank(s) failed", bad);
  }
  return 0;
}
