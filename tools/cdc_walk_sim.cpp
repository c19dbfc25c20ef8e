// tools/cdc_walk_sim.cpp -- CPU simulation behind the FastCDC walk path's design (DESIGN §4 "W + X"):
// on 1 GiB of splitmix data at C5's 4096 / 8192 / 16384, the share of bytes cut_gear hashes, how
// often a chunk is cut inside the first 47 hashed positions (where W's relaxed test differs), how far
// a relaxed walk started anywhere runs before it lands on the true chain, and per-section round counts
// (mean, E[max of 64 lanes]) for section and warm-up sizes.
//   g++ -O2 -o /tmp/cdc_walk_sim tools/cdc_walk_sim.cpp && /tmp/cdc_walk_sim
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <set>
#include <algorithm>
#include <cmath>
#include "../oxen_amd/csrc/fastcdc_gear.h"
typedef uint64_t u64;
static u64 MS = 0x0000d90313530000ULL, ML = 0x0000d90103530000ULL;  // avg 8K level1
static u64 cut(const uint8_t* s, u64 len, u64 mn, u64 avg, u64 mx, bool relaxed) {
  u64 rem = len; if (rem <= mn) return rem; u64 c = avg; if (rem > mx) rem = mx; else if (rem < c) c = rem;
  u64 a0 = mn / 2 * 2, eS = c / 2 * 2, eL = rem / 2 * 2; u64 h = 0;
  for (u64 q = a0; q < eL; ++q) { h = (h << 1) + oxh::kGear[s[q]];
    if (relaxed && q < a0 + 47) continue;
    if ((h & (q < eS ? MS : ML)) == 0) return q; }
  return rem;
}
int main(int argc, char** argv) {
  u64 N = 1ull << 30; std::vector<uint8_t> d(N); u64 x = 12345;
  for (u64 i = 0; i < N; i += 8) { x += 0x9E3779B97F4A7C15ull; u64 z = x; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; z ^= z >> 31; *(u64*)&d[i] = z; }
  u64 mn = 4096, avg = 8192, mx = 16384;
  // exact chain
  std::vector<u64> ex; u64 p = 0, rolled = 0; u64 bad = 0;
  while (p < N) { ex.push_back(p); u64 c = cut(&d[p], N - p, mn, avg, mx, false); u64 r = cut(&d[p], N - p, mn, avg, mx, true); if (c != r) ++bad; rolled += (c > mn ? c - mn / 2 * 2 : 0); p += c; }
  printf("chunks %zu mean %.1f bad %llu (%.4f%%) rolled frac %.3f\n", ex.size(), (double)N / ex.size(), (unsigned long long)bad, 100.0 * bad / ex.size(), (double)rolled / N);
  std::set<u64> exs(ex.begin(), ex.end());
  // relaxed walk from random starts: distance (bytes) until it lands on an exact-chain start
  srand(7); std::vector<u64> dist; int never = 0;
  for (int t = 0; t < 20000; ++t) { u64 s = (u64)rand() * 4096 % (N - (4 << 20)); u64 q = s; int k = 0;
    while (!exs.count(q) && k < 200) { q += cut(&d[q], N - q, mn, avg, mx, true); ++k; }
    if (k >= 200) { ++never; continue; } dist.push_back(q - s); }
  std::sort(dist.begin(), dist.end());
  auto pct = [&](double f) { return dist[(size_t)(f * (dist.size() - 1))]; };
  printf("landing distance: p50 %llu p90 %llu p99 %llu p999 %llu max %llu never %d\n", (unsigned long long)pct(.5), (unsigned long long)pct(.9), (unsigned long long)pct(.99), (unsigned long long)pct(.999), (unsigned long long)dist.back(), never);
  for (u64 W : {0ull, 16384ull, 32768ull, 65536ull}) {
  for (u64 S : {704ull << 10, 352ull << 10}) {
    std::vector<double> rs;
    for (u64 s0 = 0; s0 + S + 65536 < N; s0 += S) {
      u64 q = s0 > W ? s0 - W : 0; u64 rounds = 0;
      while (q < s0 + S) { u64 c = cut(&d[q], N - q, mn, avg, mx, true); u64 ls = (q + mn / 2 * 2) & ~127ull; u64 e = q + c;
        rounds += (e > ls ? (e - ls + 127) / 128 : 0) + 1; q = e; }
      rs.push_back((double)rounds); }
    double m = 0, v = 0; for (double r : rs) m += r; m /= rs.size(); for (double r : rs) v += (r - m) * (r - m); v = sqrt(v / rs.size());
    // expected max of 64 (sample)
    double em = 0; int groups = 0; for (size_t i = 0; i + 64 <= rs.size(); i += 64) { em += *std::max_element(rs.begin() + i, rs.begin() + i + 64); ++groups; }
    em /= groups;
    printf("warmup %llu sec %llu KiB: rounds mean %.0f sd %.0f (%.2f%%) E[max64] %.0f (+%.1f%%) ideal %.0f -> eff bytes/round %.1f\n", (unsigned long long)W, (unsigned long long)(S >> 10), m, v, 100 * v / m, em, 100 * (em / m - 1), S * 0.609 / 128, (double)S / em);
  } }
  return 0;
}
