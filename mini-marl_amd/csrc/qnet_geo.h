// Q-network parameter geometry: canonical flat layout + MFMA fragment image layout.
#pragma once
#include "common.h"
#include "minimarl.h"

namespace mm {

// Canonical flat layout (element offsets), see include/minimarl.h.
struct QnetOffsets {
  int64_t W1, b1, W2, b2, Wih, Whh, bih, bhh, Wq, bq, total;
};

// Per-agent packed fragment image (element offsets inside one agent's image).
struct QnetGeo {
  int KD;  // ceil(D/32)
  int64_t off_l1, off_l2, off_ih, off_hh, off_q;
  int64_t off_b1, off_b2, off_brz, off_bin, off_bhn, off_bq;
  int64_t agent_stride;
};

// Compile-time view of QnetGeo for the kernel instantiations (must match qnet_geometry).
template <int F1, int G, int H, int AB>
struct QnetCGeo {
  static constexpr int RB1 = F1 / 32, RB2 = G / 32, HB = H / 32;
  static constexpr int off_l2 = 0;
  static constexpr int off_ih = off_l2 + RB2 * RB1 * 1024;
  static constexpr int off_hh = off_ih + 3 * HB * RB2 * 1024;
  static constexpr int off_q = off_hh + 3 * HB * HB * 1024;
  static constexpr int off_b1 = off_q + AB * HB * 1024;
  static constexpr int off_b2 = off_b1 + RB1 * 32;
  static constexpr int off_brz = off_b2 + RB2 * 32;
  static constexpr int off_bin = off_brz + 2 * HB * 32;
  static constexpr int off_bhn = off_bin + HB * 32;
  static constexpr int off_bq = off_bhn + HB * 32;
  static constexpr int off_l1 = off_bq + AB * 32;
};

inline int qnet_check(const mm_qnet_dims* d) {
  MM_REQUIRE(d, "qnet: null dims");
  MM_REQUIRE(d->n_agents >= 1 && d->obs_dim >= 1 && d->n_actions >= 1 && d->n_actions <= 64,
             "qnet: bad dims N=%d D=%d A=%d", d->n_agents, d->obs_dim, d->n_actions);
  MM_REQUIRE(d->f1 % 32 == 0 && d->g % 32 == 0 && d->h % 32 == 0 && d->f1 > 0 && d->g > 0 && d->h > 0,
             "qnet: F1/G/H must be positive multiples of 32 (got %d/%d/%d)", d->f1, d->g, d->h);
  return MM_OK;
}

inline int qnet_offsets(const mm_qnet_dims* d, QnetOffsets* o) {
  int rc = qnet_check(d);
  if (rc) return rc;
  const int64_t N = d->n_agents, D = d->obs_dim, F1 = d->f1, G = d->g, H = d->h, A = d->n_actions;
  int64_t c = 0;
  o->W1 = c; c += N * F1 * D;
  o->b1 = c; c += N * F1;
  o->W2 = c; c += N * G * F1;
  o->b2 = c; c += N * G;
  o->Wih = c; c += N * 3 * H * G;
  o->Whh = c; c += N * 3 * H * H;
  o->bih = c; c += N * 3 * H;
  o->bhh = c; c += N * 3 * H;
  o->Wq = c; c += N * A * H;
  o->bq = c; c += N * A;
  o->total = c;
  return MM_OK;
}

inline int qnet_geometry(const mm_qnet_dims* d, QnetGeo* g, QnetOffsets* o) {
  int rc = qnet_offsets(d, o);
  if (rc) return rc;
  const int64_t RB1 = d->f1 / 32, RB2 = d->g / 32, HB = d->h / 32, AB = (d->n_actions + 31) / 32;
  g->KD = (d->obs_dim + 31) / 32;
  // Everything whose size is fixed by (F1, G, H, A) first, layer 1 (size depends on D) last,
  // so the kernels address all post-layer-1 fragments with compile-time offsets (QnetCGeo).
  int64_t c = 0;
  g->off_l2 = c; c += RB2 * RB1 * 1024;
  g->off_ih = c; c += 3 * HB * RB2 * 1024;
  g->off_hh = c; c += 3 * HB * HB * 1024;
  g->off_q = c; c += AB * HB * 1024;
  g->off_b1 = c; c += RB1 * 32;
  g->off_b2 = c; c += RB2 * 32;
  g->off_brz = c; c += 2 * HB * 32;
  g->off_bin = c; c += HB * 32;
  g->off_bhn = c; c += HB * 32;
  g->off_bq = c; c += AB * 32;
  g->off_l1 = c; c += RB1 * g->KD * 1024;
  g->agent_stride = (c + 255) & ~int64_t(255);  // whole 1 KiB chunks (LDS-DMA staging)
  return MM_OK;
}

}  // namespace mm
