/*
 * zb_host_selftest.cpp — host-sanitizer driver for zb_host.cpp (host code under
 * -fsanitize=address,undefined; built by csrc/sanitize.mk, run by tests/test_sanitizers.py).
 *
 *   zb_host_selftest <model.bin> <config.bin> [mutations]
 *
 * The model / config are the raw ZbModel / ZbEnvConfig bytes compile_model() and default_config()
 * produce. The driver validates them (expects ZB_OK), builds the team topology, and then feeds
 * check_model / check_cfg `mutations` corrupted copies: one to four 32-bit words of the struct
 * replaced by small integers, boundary values or random bits (deterministic xorshift). Every
 * copy that passes validation is handed to build_topology, which must then stay inside the
 * model's arrays: an out-of-bounds index the validation let through is an ASan / UBSan report
 * (-fsanitize=bounds sees the fixed-size member arrays). Prints one summary line.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "zb_host.h"

static bool read_file(const char* path, void* dst, size_t bytes) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  size_t got = fread(dst, 1, bytes, f);
  int extra = fgetc(f);
  fclose(f);
  return got == bytes && extra == EOF;
}

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s model.bin config.bin [mutations]\n", argv[0]);
    return 2;
  }
  const long mutations = argc > 3 ? atol(argv[3]) : 20000;
  ZbModel* model = new ZbModel;
  ZbEnvConfig cfg;
  if (!read_file(argv[1], model, sizeof *model) || !read_file(argv[2], &cfg, sizeof cfg)) {
    fprintf(stderr, "cannot read %s / %s as ZbModel (%zu B) / ZbEnvConfig (%zu B)\n", argv[1], argv[2],
            sizeof(ZbModel), sizeof(ZbEnvConfig));
    return 2;
  }
  if (zb::check_model(model) != ZB_OK || zb::check_cfg(&cfg) != ZB_OK) {
    fprintf(stderr, "the unmodified model / config fail validation: %s\n", zb_last_error());
    return 1;
  }
  static int32_t topo[zb::TP_NF][zb::TOPO_LANES];
  zb::build_topology(model, topo);
  long roots = 0;
  for (int l = 0; l < zb::TOPO_LANES; l++) roots += topo[zb::TP_DFREE][l];
  if (roots != 6) {
    fprintf(stderr, "topology: %ld free-joint dof lanes, expected 6\n", roots);
    return 1;
  }
  ZbEnvConfig dflt;
  zb_default_config(&dflt);
  if (memcmp(&dflt, &cfg, sizeof cfg) != 0) fprintf(stderr, "note: config differs from zb_default_config\n");

  const size_t words = sizeof(ZbModel) / 4;
  const int32_t specials[] = {-1, 0, 1, 2, 5, 6, 7, 12, 13, 25, 26, 27, 31, 32, 33, 40, 64, 127, 255, 1000,
                              -1000, 0x7fffffff, (int32_t)0x80000000};
  const int nspecial = (int)(sizeof specials / sizeof specials[0]);
  long accepted = 0, rejected = 0;
  ZbModel* m = new ZbModel;
  for (long it = 0; it < mutations; it++) {
    memcpy(m, model, sizeof *m);
    uint32_t* w = reinterpret_cast<uint32_t*>(m);
    const int k = 1 + (int)(next_u64() % 4);
    for (int j = 0; j < k; j++) {
      /* keep the header (magic, version, struct_bytes) mostly intact so the deep checks run */
      size_t at = (size_t)(next_u64() % words);
      if (at < 3 && (next_u64() & 7)) at = 3 + (size_t)(next_u64() % (words - 3));
      const uint64_t r = next_u64();
      switch (r % 3) {
        case 0: w[at] = (uint32_t)specials[(r >> 8) % nspecial]; break;
        case 1: w[at] = (uint32_t)((int32_t)((r >> 8) % 80) - 8); break;
        default: w[at] = (uint32_t)(r >> 16); break;
      }
    }
    if (zb::check_model(m) == ZB_OK) {
      accepted++;
      zb::build_topology(m, topo);
    } else {
      rejected++;
    }
    ZbEnvConfig c = cfg;
    uint32_t* cw = reinterpret_cast<uint32_t*>(&c);
    cw[next_u64() % (sizeof c / 4)] = (uint32_t)next_u64();
    (void)zb::check_cfg(&c);
  }
  printf("zb_host_selftest ok: %ld mutations, %ld accepted, %ld rejected, words %zu\n", mutations, accepted,
         rejected, words);
  delete m;
  delete model;
  return 0;
}
