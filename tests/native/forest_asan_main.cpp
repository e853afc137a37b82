// Standalone driver for the host forest engine under AddressSanitizer + UBSan
// (tests/test_sanitizers.py builds it with -fsanitize=address,undefined and runs it).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../csrc/forest_common.hpp"

using atef::ForestParams;
extern "C" int atecpu_forest_fit(const ForestParams*, const uint8_t*, const uint8_t*,
                                 const int64_t*, const int64_t*, int, int32_t*, int32_t*,
                                 int32_t*, double*, int32_t*, uint8_t*, int64_t*, int);
extern "C" int atecpu_forest_predict(const ForestParams*, const uint8_t*, int, int, int,
                                     const int32_t*, const int32_t*, const int32_t*,
                                     const double*, const uint8_t*, const int64_t*, double*, int,
                                     double*, int);

int main() {
  const int n = 600, p = 7, ntree = 8;
  std::vector<uint8_t> Xb((size_t)p * n), y(n);
  std::vector<int64_t> r1(n), r2(n);
  uint32_t s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s >> 8; };
  for (auto& v : Xb) v = (uint8_t)(rnd() % 200);
  for (int i = 0; i < n; ++i) {
    y[i] = Xb[i] > 100;
    r1[i] = (int64_t)(rnd() % 1000) * 4294967LL - 2147483648LL;
    r2[i] = (int64_t)(rnd() % 1000) * 4294967LL - 2147483648LL;
  }
  for (int kind = 0; kind < 3; ++kind) {
    ForestParams fp{};
    fp.kind = kind;
    fp.sampling = kind == 0 ? 0 : 1;
    fp.ntree = ntree;
    fp.mtry = 3;
    fp.min_node = kind == 0 ? 1 : 5;
    fp.honesty = kind != 0;
    fp.group = kind == 0 ? 1 : 2;
    fp.mtry_poisson = kind != 0;
    fp.alpha = kind == 0 ? 0.0 : 0.05;
    fp.sample_fraction = 0.5;
    fp.pois0 = 0.049787068367863944;
    fp.seed = 7;
    fp.p = p;
    fp.n = n;
    fp.t0 = 0;
    const int cap = 2 * n + 1;
    std::vector<int32_t> feat((size_t)ntree * cap), thr(feat.size()), left(feat.size()), nn(ntree);
    std::vector<double> val(feat.size());
    std::vector<uint8_t> inbag((size_t)ntree * n);
    std::vector<int64_t> est(fp.sampling == 1 ? feat.size() * 5 : 0);
    int rc = atecpu_forest_fit(&fp, Xb.data(), y.data(), r1.data(), r2.data(), cap, feat.data(),
                               thr.data(), left.data(), val.data(), nn.data(), inbag.data(),
                               est.empty() ? nullptr : est.data(), 2);
    if (rc) return 10 + kind;
    const int width = kind == 2 ? 4 : 1;
    std::vector<double> state((size_t)10 * n, 0.0), out((size_t)n * width);
    rc = atecpu_forest_predict(&fp, Xb.data(), n, 1, cap, feat.data(), thr.data(), left.data(),
                               val.data(), inbag.data(), est.empty() ? nullptr : est.data(),
                               state.data(), 7, out.data(), 2);
    if (rc) return 20 + kind;
    std::printf("kind %d ok: nodes[0]=%d out[0]=%g\n", kind, nn[0], out[0]);
  }
  return 0;
}
