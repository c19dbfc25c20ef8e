// tools/cdc_walk_emu.cpp -- CPU emulation of W's per-lane state machine (cdc_walk_scan_kernel: lines,
// bubbles, round masks, the group resolve, begin-chunk rules) and X's stitch, on 64 MiB of splitmix
// data at C5's parameters, checked against a direct cut_gear walk. Written to test the design before the
// first GPU run; the GPU path itself is checked by tests/test_fastcdc.py and bench_fastcdc --check-all.
//   g++ -O2 -o /tmp/cdc_walk_emu tools/cdc_walk_emu.cpp && /tmp/cdc_walk_emu
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "../oxen_amd/csrc/fastcdc_gear.h"
typedef uint64_t u64; typedef uint32_t u32;
static u64 MS, ML;
static u64 MN = 4096, AVG = 8192, MX = 16384;
static const u32 kFull = 0xFFFFFFFFu;
static u64 cut_exact(const uint8_t* s, u64 len) {
  u64 rem = len; if (rem <= MN) return rem; u64 c = AVG; if (rem > MX) rem = MX; else if (rem < c) c = rem;
  u64 a0 = MN & ~1ull, eS = c & ~1ull, eL = rem & ~1ull; u64 h = 0;
  for (u64 q = a0; q < eL; ++q) { h = (h << 1) + oxh::kGear[s[q]]; if ((h & (q < eS ? MS : ML)) == 0) return q; }
  return rem;
}
struct Lane { u32 cs, lo, tS, tL, cutm, mS, mE, mF, n; bool done; std::vector<u32> out; };
static void begin(Lane& L) {
  for (;;) {
    if (L.cs >= L.mS) { L.out.push_back(L.cs - L.mS); ++L.n; if ((L.cs >= L.mE && L.n > 1) || L.cs >= L.mF) { L.done = true; return; } }
    u32 len = L.mF - L.cs; if (len <= MN) { L.cs += len; continue; }
    u32 rem = len > MX ? MX : len; u32 center = AVG; if (len <= MX && len < center) center = len;
    u32 a0 = MN & ~1u; L.lo = L.cs + a0 + 47; L.tS = L.cs + (center & ~1u); L.tL = L.cs + (rem & ~1u); L.cutm = L.cs + rem;
    if (L.lo >= L.tL) { L.cs = L.cutm; continue; }
    return;
  }
}
int main() {
  u64 N = 64ull << 20; std::vector<uint8_t> d(N + 4096); u64 x = 99;
  for (u64 i = 0; i < N; i += 8) { x += 0x9E3779B97F4A7C15ull; u64 z = x; z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; z ^= z >> 31; *(u64*)&d[i] = z; }
  MS = 0x0000d90313530000ULL; ML = 0x0000d90103530000ULL;
  u64 ms64 = MS << 16, ml64 = ML << 16; u32 ms = ms64 >> 32, ml = ml64 >> 32, mc = ms & ml;
  // oracle chain
  std::vector<u64> ex; for (u64 p = 0; p < N;) { ex.push_back(p); p += cut_exact(&d[p], N - p); }
  u64 SEC = 704 << 10, WU = 2 * MX; u64 nsec = (N + SEC - 1) / SEC;
  std::vector<std::vector<u32>> spec(nsec);
  u64 rounds_total = 0, max_rounds = 0;
  for (u64 sc = 0; sc < nsec; ++sc) {
    u64 S = sc * SEC, E = std::min(N, S + SEC), W0 = S > WU ? S - WU : 0;
    Lane L{}; L.mS = S; L.mE = E; L.mF = std::min<u64>(N, S + SEC + 2 * MX + 4096); L.cs = W0; L.done = false; L.n = 0;
    begin(L);
    u32 a0 = MN & ~1u; u32 NL = L.done ? 0xFFFFFF00u : ((L.cs + a0) & ~127u);
    u32 RL = NL; bool RV = !L.done; if (!L.done) NL += 128;
    u64 h = 0; u64 rounds = 0;
    while (!L.done) {
      ++rounds;
      u32 CL = RL; bool CV = RV && !L.done; RL = L.done ? 0xFFFFFF00u : NL; RV = !L.done; if (!L.done) NL += 128;
      u32 m; if (!CV || CL + 128 <= L.lo) m = kFull; else if (CL + 128 <= L.tS) m = ms; else if (CL >= L.tS) m = ml; else m = mc;
      bool cut_now = false;
      for (int g = 0; g < 8; ++g) {
        u32 hh[16]; u32 anyz = 0xFFFFFFFFu;
        for (int j = 0; j < 16; ++j) { u64 pos = CL + 16 * g + j; uint8_t b = pos < d.size() ? d[pos] : 0; h = (h << 1) + (oxh::kGear[b] << 16); hh[j] = h >> 32; anyz = std::min(anyz, hh[j] & m); }
        if (anyz == 0) {
          u32 gpos = CL + 16 * g; u32 bits = 0; for (int j = 0; j < 16; ++j) bits |= ((hh[j] & m) == 0 ? 1u : 0u) << j;
          while (bits) { int j = __builtin_ctz(bits); bits &= bits - 1; u32 p = gpos + j;
            if (p < L.lo || p >= L.tL) continue;
            if (m == mc) { if ((hh[j] & (p < L.tS ? ms : ml)) != 0) continue; }
            L.cs = p; begin(L); if (!L.done) NL = (L.cs + a0) & ~127u; RV = false; m = kFull; cut_now = true; break; }
        }
      }
      if (CV && !cut_now && CL + 128 >= L.tL) { L.cs = L.cutm; begin(L); if (!L.done) NL = (L.cs + a0) & ~127u; RV = false; }
    }
    spec[sc] = L.out; rounds_total += rounds; max_rounds = std::max(max_rounds, rounds);
  }
  // relaxed-chain check: each spec entry k -> entry k+1 must be the relaxed cut (no truncated tests)
  u64 bad_relax = 0, chunks = 0;
  for (u64 sc = 0; sc < nsec; ++sc) { u64 S = sc * SEC; auto& v = spec[sc];
    for (size_t k = 0; k + 1 < v.size(); ++k) { u64 c = S + v[k]; u64 len = N - c; u64 rem = len; u64 want;
      if (rem <= MN) want = rem; else { u64 cen = AVG; if (rem > MX) rem = MX; else if (rem < cen) cen = rem; u64 a0 = MN & ~1ull, eS = cen & ~1ull, eL = rem & ~1ull; u64 hh = 0; want = rem;
        for (u64 q = a0; q < eL; ++q) { hh = (hh << 1) + oxh::kGear[d[c + q]]; if (q >= a0 + 47 && (hh & (q < eS ? MS : ML)) == 0) { want = q; break; } } }
      ++chunks; if (S + v[k + 1] != c + want) { if (bad_relax < 5) printf("relax mismatch sec %llu k %zu: got %llu want %llu\n", (unsigned long long)sc, k, (unsigned long long)(v[k+1]), (unsigned long long)(c + want - S)); ++bad_relax; } } }
  printf("sections %llu chunks %llu relaxed-mismatch %llu rounds mean %.0f max %llu\n", (unsigned long long)nsec, (unsigned long long)chunks, (unsigned long long)bad_relax, (double)rounds_total / nsec, (unsigned long long)max_rounds);
  // X: exact walk stitched from the lists
  std::vector<u64> got; u64 e = 0;
  for (u64 sc = 0; sc < nsec; ++sc) { u64 S = sc * SEC, E = std::min(N, S + SEC); auto& v = spec[sc]; u64 p = e;
    auto lookup = [&](u64 pos) -> long { auto it = std::lower_bound(v.begin(), v.end(), (u32)(pos - S)); return (it != v.end() && *it == (u32)(pos - S)) ? long(it - v.begin()) : -1; };
    long j = lookup(p);
    while (p < E) { got.push_back(p);
      if (j >= 0 && (size_t)j + 1 < v.size()) { u64 tc = ~0ull; // trunc check of p
          u64 len = N - p; if (len > MN) { u64 rem = len > MX ? MX : len; u64 cen = AVG; if (len <= MX && len < cen) cen = len; u64 a0 = MN & ~1ull, eS = cen & ~1ull, eL = rem & ~1ull; u64 tend = std::min(a0 + 47, eL); u64 hh = 0;
            for (u64 q = a0; q < a0 + 47; ++q) { hh = (hh << 1) + oxh::kGear[d[p + q]]; if (q < tend && (hh & (q < eS ? MS : ML)) == 0) { tc = p + q; break; } } }
          if (tc == ~0ull) { ++j; p = S + v[j]; continue; } p = tc; }
      else p += cut_exact(&d[p], N - p);
      j = lookup(p); }
    e = p; }
  printf("exact chunks %zu got %zu equal %d\n", ex.size(), got.size(), (int)(ex == got));
  return 0;
}
