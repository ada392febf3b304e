// Host check of the fused rollout step's per-env pieces (mini-marl_amd/csrc/fused_env.h: grid packing,
// obs masks / features, dynamics) against oracle/env.py records written by tests/test_fused_env_host.py.
// Built and run by that test on the CPU (no GPU): exit 0 and "OK <n>" when every value is bit-identical.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fused_env.h"

using mm::FusedEnv;

static int fail(const char* what, int rec, int e, int a, int f, double got, double want) {
  std::printf("MISMATCH %s record %d env %d agent %d item %d: got %.9g want %.9g\n", what, rec, e, a, f, got, want);
  return 1;
}

template <class T>
static void rd(FILE* fp, T* dst, size_t n) {
  if (std::fread(dst, sizeof(T), n, fp) != n) {
    std::printf("short read\n");
    std::exit(2);
  }
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* fp = std::fopen(argv[1], "rb");
  if (!fp) return 2;
  int32_t hdr[8];
  rd(fp, hdr, 8);
  const int E = hdr[0], N = hdr[1], R = hdr[2], C = hdr[3], D = hdr[4], full = hdr[5], max_steps = hdr[6],
            nrec = hdr[7];
  float fh[3];
  rd(fp, fh, 3);
  const int RC = R * C, NPW = (RC + 15) >> 4;
  FusedEnv ev{};
  ev.E = E;
  ev.N = N;
  ev.R = R;
  ev.C = C;
  ev.D = D;
  ev.max_steps = max_steps;
  ev.full_obs = full;
  ev.step_cost = fh[0];
  ev.inv_r = fh[1];
  ev.inv_c = fh[2];
  std::vector<int32_t> ipos(N * 2);
  std::vector<int8_t> igrid(RC);
  std::vector<float> iobs((size_t)N * D);
  rd(fp, ipos.data(), ipos.size());
  rd(fp, igrid.data(), igrid.size());
  rd(fp, iobs.data(), iobs.size());
  std::vector<int32_t> pos((size_t)E * N * 2), pos2((size_t)E * N * 2), act((size_t)E * N), steps(E), apples(E);
  std::vector<int8_t> grid((size_t)E * RC + 16), grid2((size_t)E * RC);
  std::vector<float> obs((size_t)E * N * D), obs2((size_t)E * N * D), rew((size_t)E * N);
  std::vector<uint8_t> done(E);
  // LDS-shaped scratch: items FS_ENVS apart, env 0
  std::vector<uint16_t> sp(8 * mm::FS_ENVS);
  std::vector<uint64_t> sm(4 * mm::FS_ENVS);
  long checked = 0;
  for (int rec = 0; rec < nrec; ++rec) {
    rd(fp, pos.data(), pos.size());
    rd(fp, grid.data(), (size_t)E * RC);
    rd(fp, steps.data(), steps.size());
    rd(fp, apples.data(), apples.size());
    rd(fp, obs.data(), obs.size());
    rd(fp, act.data(), act.size());
    rd(fp, obs2.data(), obs2.size());
    rd(fp, rew.data(), rew.size());
    rd(fp, done.data(), done.size());
    rd(fp, pos2.data(), pos2.size());
    rd(fp, grid2.data(), grid2.size());
    for (int e = 0; e < E; ++e) {
      uint32_t g[8] = {0};
      for (int pw = 0; pw < NPW; ++pw) g[pw] = mm::fs_load_word(grid.data() + (size_t)e * RC, RC, pw);
      for (int i = 0; i < RC; ++i)
        if (mm::fs_cell(g, 1, i) != grid[(size_t)e * RC + i]) return fail("packed grid", rec, e, -1, i, mm::fs_cell(g, 1, i), grid[(size_t)e * RC + i]);
      int pr[8], pc[8], ak[8];
      for (int j = 0; j < 8; ++j) {
        pr[j] = j < N ? pos[((size_t)e * N + j) * 2] : -100;
        pc[j] = j < N ? pos[((size_t)e * N + j) * 2 + 1] : -100;
        ak[j] = j < N ? act[(size_t)e * N + j] : 4;
      }
      for (int a = 0; a < N; ++a) {   // obs of the state before the step
        mm::fs_publish(ev, pr, pc, g, 1, a, sp.data(), sm.data(), mm::FS_ENVS);
        for (int f = 0; f < D; ++f) {
          const float got = mm::fs_feature(ev, sp.data(), sm.data(), nullptr, nullptr, 0, false, a, f);
          const float want = obs[((size_t)e * N + a) * D + f];
          if (std::memcmp(&got, &want, 4)) return fail("obs", rec, e, a, f, got, want);
          ++checked;
        }
      }
      int st = steps[e], ap = apples[e];
      float rw[8];
      const bool dn = mm::fs_dynamics(ev, pr, pc, ak, g, 1, st, ap, rw);
      if (dn != (done[e] != 0)) return fail("done", rec, e, -1, -1, dn, done[e]);
      for (int k = 0; k < N; ++k) {
        if (std::memcmp(&rw[k], &rew[(size_t)e * N + k], 4)) return fail("rew", rec, e, k, -1, rw[k], rew[(size_t)e * N + k]);
        if (pr[k] != pos2[((size_t)e * N + k) * 2] || pc[k] != pos2[((size_t)e * N + k) * 2 + 1])
          return fail("pos", rec, e, k, -1, pr[k] * 256 + pc[k], pos2[((size_t)e * N + k) * 2] * 256 + pos2[((size_t)e * N + k) * 2 + 1]);
      }
      for (int i = 0; i < RC; ++i)
        if (mm::fs_cell(g, 1, i) != grid2[(size_t)e * RC + i]) return fail("next grid", rec, e, -1, i, mm::fs_cell(g, 1, i), grid2[(size_t)e * RC + i]);
      if ((RC & 3) == 0)   // the kernel's dword grid write-back
        for (int i = 0; i < RC; i += 4) {
          const uint32_t w = mm::fs_unpack4((g[i >> 4] >> (2 * (i & 15))) & 0xFFu);
          uint32_t want;
          std::memcpy(&want, grid2.data() + (size_t)e * RC + i, 4);
          if (w != want) return fail("unpack", rec, e, -1, i, w, want);
        }
      for (int a = 0; a < N; ++a) {   // terminal next obs
        mm::fs_publish(ev, pr, pc, g, 1, a, sp.data(), sm.data(), mm::FS_ENVS);
        for (int f = 0; f < D; ++f) {
          const float got = mm::fs_feature(ev, sp.data(), sm.data(), nullptr, nullptr, 0, false, a, f);
          const float want = obs2[((size_t)e * N + a) * D + f];
          if (std::memcmp(&got, &want, 4)) return fail("next obs", rec, e, a, f, got, want);
          ++checked;
        }
      }
    }
  }
  // reset obs from the initial state's masks (the kernel's s_ipos / s_imask path)
  {
    uint32_t g[8] = {0};
    for (int pw = 0; pw < NPW; ++pw) g[pw] = mm::fs_load_word(igrid.data(), RC, pw);
    int pr[8], pc[8];
    uint16_t ip[8];
    for (int j = 0; j < 8; ++j) {
      pr[j] = j < N ? ipos[j * 2] : -100;
      pc[j] = j < N ? ipos[j * 2 + 1] : -100;
      ip[j] = (uint16_t)(j < N ? ((pr[j] << 8) | pc[j]) : 0);
    }
    for (int a = 0; a < N; ++a) {
      uint64_t im[4] = {0, 0, 0, 0};
      uint16_t junk[8];
      mm::fs_publish(ev, pr, pc, g, 1, a, junk, im, 1);
      for (int f = 0; f < D; ++f) {
        const float got = mm::fs_feature(ev, nullptr, nullptr, ip, im, 0, true, a, f);
        const float want = iobs[(size_t)a * D + f];
        if (std::memcmp(&got, &want, 4)) return fail("reset obs", -1, -1, a, f, got, want);
        ++checked;
      }
    }
  }
  std::printf("OK %ld\n", checked);
  return 0;
}
