// Standalone driver for the host forest engine under AddressSanitizer + UBSan
// (tests/test_sanitizers.py builds it with -fsanitize=address,undefined and runs it).
// Covers the 256-bin engine (randomForest bootstrap, grf little bags of 2 and of 1), the
// exact-split engine (uint16 value ranks: randomForest kinds 0/1, grf regression with
// ci.group.size 1, honest causal little bags), both predictors and the variance debiaser.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../csrc/forest_common.hpp"

using atef::ForestParams;
extern "C" int atecpu_forest_fit(const ForestParams*, const uint8_t*, const uint8_t*,
                                 const int64_t*, const int64_t*, int, int32_t*, int32_t*,
                                 int32_t*, double*, int32_t*, uint8_t*, int64_t*, int);
extern "C" int atecpu_forest_fit_exact(const ForestParams*, const uint16_t*, const double*, int,
                                       const int32_t*, const uint8_t*, const int64_t*,
                                       const int64_t*, int, int32_t*, int32_t*, int32_t*, double*,
                                       int32_t*, uint8_t*, int64_t*, int);
extern "C" int atecpu_forest_predict(const ForestParams*, const uint8_t*, int, int, int,
                                     const int32_t*, const int32_t*, const int32_t*,
                                     const double*, const uint8_t*, const int64_t*, int64_t*, int,
                                     double*, int);
extern "C" int atecpu_forest_predict16(const ForestParams*, const uint16_t*, int, int, int,
                                       const int32_t*, const int32_t*, const int32_t*,
                                       const double*, const uint8_t*, const int64_t*, int64_t*,
                                       int, double*, int);
extern "C" double atecpu_grf_debias(double, double, double);

namespace {

const int n = 600, p = 7, ntree = 8;

ForestParams params(int kind, int sampling, int group) {
  ForestParams fp{};
  fp.kind = kind;
  fp.sampling = sampling;
  fp.ntree = ntree;
  fp.mtry = 3;
  fp.min_node = sampling == 0 ? 1 : 5;
  fp.honesty = sampling == 1;
  fp.group = group;
  fp.mtry_poisson = sampling == 1;
  fp.alpha = sampling == 0 ? 0.0 : 0.05;
  fp.sample_fraction = 0.5;
  fp.pois0 = std::exp(-3.0);
  fp.seed = 7;
  fp.p = p;
  fp.n = n;
  fp.t0 = 0;
  return fp;
}

struct Trees {
  std::vector<int32_t> feat, thr, left, nn;
  std::vector<double> val;
  std::vector<uint8_t> inbag;
  std::vector<int64_t> est;
  int cap;
  explicit Trees(const ForestParams& fp) : cap(2 * n + 1) {
    feat.resize((size_t)ntree * cap);
    thr.resize(feat.size());
    left.resize(feat.size());
    val.resize(feat.size());
    nn.resize(ntree);
    inbag.resize((size_t)ntree * n);
    est.resize(fp.sampling == 1 ? feat.size() * 5 : 0);
  }
  int64_t* e() { return est.empty() ? nullptr : est.data(); }
};

}  // namespace

int main() {
  std::vector<uint8_t> Xb((size_t)p * n), y(n);
  std::vector<uint16_t> Xr((size_t)p * n);
  std::vector<int64_t> r1(n), r2(n);
  uint32_t s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s >> 8; };
  for (auto& v : Xb) v = (uint8_t)(rnd() % 200);
  // exact mode: value ranks with a per-feature table of distinct values (few for feature 0)
  const int ldv = 300;
  std::vector<double> vals((size_t)p * ldv, INFINITY);
  std::vector<int32_t> nval(p);
  for (int j = 0; j < p; ++j) {
    nval[j] = j == 0 ? 3 : ldv;
    for (int v = 0; v < nval[j]; ++v) vals[(size_t)j * ldv + v] = 0.5 * v - 7.0;
    for (int i = 0; i < n; ++i) Xr[(size_t)j * n + i] = (uint16_t)(rnd() % nval[j]);
  }
  for (int i = 0; i < n; ++i) {
    y[i] = Xb[i] > 100;
    r1[i] = (int64_t)(rnd() % 1000) * 4294967LL - 2147483648LL;
    r2[i] = (int64_t)(rnd() % 1000) * 4294967LL - 2147483648LL;
  }
  struct Case { int kind, sampling, group; bool exact; };
  const Case cases[] = {{0, 0, 1, false}, {1, 1, 2, false}, {2, 1, 2, false}, {1, 1, 1, false},
                        {0, 0, 1, true},  {1, 0, 1, true},  {1, 1, 1, true},  {2, 1, 2, true}};
  int ci = 0;
  for (const Case& c : cases) {
    const ForestParams fp = params(c.kind, c.sampling, c.group);
    Trees tr(fp);
    const int rc = c.exact
        ? atecpu_forest_fit_exact(&fp, Xr.data(), vals.data(), ldv, nval.data(), y.data(),
                                  r1.data(), r2.data(), tr.cap, tr.feat.data(), tr.thr.data(),
                                  tr.left.data(), tr.val.data(), tr.nn.data(), tr.inbag.data(),
                                  tr.e(), 2)
        : atecpu_forest_fit(&fp, Xb.data(), y.data(), r1.data(), r2.data(), tr.cap,
                            tr.feat.data(), tr.thr.data(), tr.left.data(), tr.val.data(),
                            tr.nn.data(), tr.inbag.data(), tr.e(), 2);
    if (rc) return 10 + ci;
    const int width = c.kind == 2 ? 4 : 1;
    std::vector<int64_t> state((size_t)10 * n, 0);
    std::vector<double> out((size_t)n * width);
    const int rp = c.exact
        ? atecpu_forest_predict16(&fp, Xr.data(), n, 1, tr.cap, tr.feat.data(), tr.thr.data(),
                                  tr.left.data(), tr.val.data(), tr.inbag.data(), tr.e(),
                                  state.data(), 7, out.data(), 2)
        : atecpu_forest_predict(&fp, Xb.data(), n, 1, tr.cap, tr.feat.data(), tr.thr.data(),
                                tr.left.data(), tr.val.data(), tr.inbag.data(), tr.e(),
                                state.data(), 7, out.data(), 2);
    if (rp) return 30 + ci;
    std::printf("case %d (kind %d sampling %d group %d exact %d) ok: nodes[0]=%d out[0]=%g\n", ci,
                c.kind, c.sampling, c.group, (int)c.exact, tr.nn[0], out[0]);
    ++ci;
  }
  double acc = 0.0;
  for (int k = 0; k < 64; ++k) acc += atecpu_grf_debias(0.1 * k, 3.0 - 0.05 * k, 2.0 + k);
  if (!(acc > 0.0) || !std::isfinite(acc)) return 50;
  std::printf("debias ok: %g\n", acc);
  return 0;
}
