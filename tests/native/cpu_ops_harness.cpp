// Host-side sanitizer harness: the CPU twins of the codec
// kernels (csrc/cpu_ops.cpp) built with -fsanitize=address,undefined and run
// on random inputs with boundary geometries (tails, one row, many blocks,
// k = 0 / k = n).  Every result is also checked against a brute-force
// reference here, so the run exercises real work, not just allocation.
// Built and run by tests/test_sanitizers.py (scripts/sanitize_host.sh).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "cpu_ops.h"

using namespace commeff;

static int g_fail = 0;
#define CHECK(c, ...)                          \
  do {                                         \
    if (!(c)) {                                \
      std::fprintf(stderr, "FAIL: " __VA_ARGS__); \
      std::fprintf(stderr, "\n");              \
      ++g_fail;                                \
    }                                          \
  } while (0)

static RowHashes make_rows(int r, std::mt19937_64& rng) {
  RowHashes h{};
  for (int j = 0; j < r; ++j) {
    h.row[j].a = rng() | 1ull;
    h.row[j].b = rng();
    h.row[j].a2 = rng() | 1ull;
    h.row[j].b2 = rng();
  }
  return h;
}

static void sketch_case(uint32_t d, uint32_t r, uint32_t c, uint32_t nb, std::mt19937_64& rng) {
  const RowHashes h = make_rows(static_cast<int>(r), rng);
  const SketchGeom g = make_geom(d, r, c, nb);
  std::vector<int32_t> blk_off(r * g.num_blocks);
  std::vector<float> blk_sign(r * g.num_blocks);
  for (auto& o : blk_off) o = static_cast<int32_t>(rng() % c);
  for (auto& s : blk_sign) s = (rng() & 1) ? 1.f : -1.f;
  std::normal_distribution<float> nd;
  std::vector<float> v(d), w(d), table(static_cast<size_t>(r) * c, 0.f), ref(table.size(), 0.f);
  for (auto& x : v) x = nd(rng);
  for (auto& x : w) x = nd(rng);
  cpu::cs_encode(table.data(), v.data(), w.data(), 0.5f, 0.25f, h, g, blk_off.data(), blk_sign.data());
  for (uint32_t i = 0; i < d; ++i)
    for (uint32_t j = 0; j < r; ++j) {
      uint32_t bk;
      float s;
      hash_coord(h.row[j], i, g, blk_off.data() + j * g.num_blocks, blk_sign.data() + j * g.num_blocks,
                 &bk, &s);
      ref[static_cast<size_t>(j) * c + bk] += s * (0.5f * v[i] + 0.25f * w[i]);
    }
  for (size_t e = 0; e < table.size(); ++e)
    CHECK(std::fabs(table[e] - ref[e]) <= 1e-3f * (1.f + std::fabs(ref[e])), "encode d=%u r=%u c=%u cell %zu",
          d, r, c, e);
  std::vector<float> est(d);
  cpu::cs_query(table.data(), est.data(), h, g, blk_off.data(), blk_sign.data());
  for (uint32_t i = 0; i < d; i += 7) {
    std::vector<float> q(r);
    for (uint32_t j = 0; j < r; ++j) {
      uint32_t bk;
      float s;
      hash_coord(h.row[j], i, g, blk_off.data() + j * g.num_blocks, blk_sign.data() + j * g.num_blocks,
                 &bk, &s);
      q[j] = s * table[static_cast<size_t>(j) * c + bk];
    }
    std::sort(q.begin(), q.end());
    CHECK(est[i] == q[(r - 1) / 2], "query d=%u i=%u", d, i);
  }
  // zero the buckets of a few coordinates
  std::vector<int64_t> idx = {0, static_cast<int64_t>(d - 1), static_cast<int64_t>(d / 2)};
  std::vector<float> vals = {1.f, 0.f, 2.f};
  std::vector<float> t2 = table;
  cpu::cs_zero_buckets(table.data(), t2.data(), idx.data(), vals.data(), 3, h, g, blk_off.data(),
                       blk_sign.data());
  (void)cpu::cs_l2estimate(table.data(), static_cast<int>(r), c);
}

static void topk_case(int64_t n, int64_t k, std::mt19937_64& rng) {
  std::normal_distribution<float> nd;
  std::vector<float> x(n);
  for (auto& e : x) e = nd(rng);
  if (n > 4) x[1] = x[3] = 7.f;  // a tie
  const int64_t kk = std::min(k, n);
  std::vector<int64_t> idx(std::max<int64_t>(kk, 1));
  std::vector<float> vals(std::max<int64_t>(kk, 1));
  cpu::topk_abs(x.data(), n, k, idx.data(), vals.data());
  std::vector<float> mag(n);
  for (int64_t i = 0; i < n; ++i) mag[i] = std::fabs(x[i]);
  std::vector<float> sorted = mag;
  std::sort(sorted.begin(), sorted.end(), std::greater<float>());
  for (int64_t t = 0; t < kk; ++t) {
    CHECK(idx[t] >= 0 && idx[t] < n, "topk idx range");
    if (t) CHECK(idx[t] > idx[t - 1], "topk ascending");
    CHECK(mag[idx[t]] >= sorted[kk - 1], "topk member n=%lld k=%lld", static_cast<long long>(n),
          static_cast<long long>(k));
  }
}

static void state_case(int64_t n, std::mt19937_64& rng) {
  std::normal_distribution<float> nd;
  std::vector<float> V(n), E(n), G(n), w(n), u(n), e(n);
  for (int64_t i = 0; i < n; ++i) {
    V[i] = nd(rng); E[i] = nd(rng); G[i] = nd(rng); w[i] = nd(rng);
  }
  cpu::momentum_ef(V.data(), E.data(), G.data(), n, 0.9f, 0.5f, 1);
  cpu::client_state(G.data(), u.data(), e.data(), n, 0.9f);
  std::vector<int32_t> last_mod(n, -1), hist(64, 0);
  std::vector<int64_t> idx;
  std::vector<float> vals;
  for (int64_t i = 0; i < n; i += 3) {
    idx.push_back(i);
    vals.push_back(G[i]);
  }
  cpu::sparse_apply(w.data(), idx.data(), vals.data(), static_cast<int64_t>(idx.size()), 0.1f, nullptr,
                    last_mod.data(), 2, hist.data());
  cpu::dense_apply(w.data(), G.data(), n, 0.1f, nullptr, last_mod.data(), 3, hist.data());
  std::vector<int32_t> thr = {0, 2, 3};
  std::vector<int64_t> cnt(3);
  cpu::count_ge(last_mod.data(), n, thr.data(), 3, cnt.data());
  CHECK(cnt[2] == n, "count_ge after dense apply");
  std::vector<float> out(n);
  cpu::axpby(out.data(), G.data(), 2.f, w.data(), -1.f, n);
  const float nrm = cpu::l2norm(out.data(), n);
  cpu::clip_noise(out.data(), n, &nrm, 1.f, 0.01f, 7, 0);
}

static void augment_case(std::mt19937_64& rng) {
  const int B = 3, H = 5, W = 7, C = 3, N = 4;
  std::vector<uint8_t> data(static_cast<size_t>(N) * H * W * C);
  for (auto& x : data) x = static_cast<uint8_t>(rng());
  std::vector<int64_t> idx = {3, 0, 2};
  const float mean[3] = {0.5f, 0.4f, 0.3f}, inv[3] = {2.f, 3.f, 4.f};
  std::vector<float> out(static_cast<size_t>(B) * H * W * C);
  cpu::augment_u8_nhwc(data.data(), idx.data(), B, H, W, C, 2, 1, mean, inv, 11, nullptr, out.data());
}

int main() {
  std::mt19937_64 rng(1234);
  sketch_case(1000, 5, 37, 1, rng);
  sketch_case(777, 1, 50, 1, rng);
  sketch_case(5003, 3, 101, 7, rng);
  sketch_case(64, 16, 8, 3, rng);
  for (int64_t n : {1, 5, 1000, 70001})
    for (int64_t k : {0, 1, 17, 1000, 70001}) topk_case(n, k, rng);
  state_case(1, rng);
  state_case(4099, rng);
  augment_case(rng);
  std::printf("%s (%d failures)\n", g_fail ? "FAILED" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
