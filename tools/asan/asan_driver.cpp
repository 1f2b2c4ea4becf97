// Host-side sanitizer driver for libimenv's C ABI (built with AddressSanitizer + UndefinedBehavior-
// Sanitizer on the host code only; tools/asan_host_check.py). No GPU is needed: it runs every path of
// the ABI that executes on the host before the first device call -- spec validation and derivation
// (validate_and_derive), the observation tables, the hipRTC source generator and compiler
// (imenv_jit_check), imenv_create up to its first allocation, and the argument checks of every entry
// point -- over the golden specs and a set of malformed ones. Replaces the reference's error paths
// (IM_env.py:203-207, MAIM_env.py:158-171, MAIM_div_env.py:505-575) with status codes, so every
// malformed spec must come back IMENV_E_INVALID / IMENV_E_UNSUPPORTED and every good one validate.
//
//   asan_driver SPECS.bin      records: int32 expect (0 valid, 1 rejected), int32 jit (compile it),
//                              char name[64], ImEnvSpec
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "imenv.h"

static int g_fail = 0;
#define CHECK(cond, ...)                                           \
  do {                                                             \
    if (!(cond)) {                                                 \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);    \
      std::fprintf(stderr, __VA_ARGS__);                           \
      std::fprintf(stderr, "\n");                                  \
      ++g_fail;                                                    \
    }                                                              \
  } while (0)

static bool rejected(int rc) { return rc == IMENV_E_INVALID || rc == IMENV_E_UNSUPPORTED; }

// argument checks that return before any device work
static void null_argument_paths() {
  ImEnv* h = nullptr;
  CHECK(imenv_create(nullptr, 16, 0, 0, &h) == IMENV_E_INVALID && !h, "create(NULL spec)");
  CHECK(imenv_reset(nullptr, nullptr, IMENV_LAYOUT_DRAW, 0, 0.0, nullptr, -1, nullptr, IMENV_F32, nullptr) ==
            IMENV_E_INVALID, "reset(NULL)");
  CHECK(imenv_step(nullptr, nullptr, IMENV_F32, nullptr, IMENV_F32, nullptr, nullptr, nullptr, nullptr) ==
            IMENV_E_INVALID, "step(NULL)");
  CHECK(imenv_get_state(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == IMENV_E_INVALID, "get_state(NULL)");
  CHECK(imenv_get_errors(nullptr, nullptr, nullptr, nullptr) == IMENV_E_INVALID, "get_errors(NULL)");
  int64_t cnt = 0;
  CHECK(imenv_debug_stamps(nullptr, nullptr, 0, &cnt) == IMENV_E_INVALID, "debug_stamps(NULL)");
  CHECK(imenv_base_stock_rollout(nullptr, nullptr, nullptr) == IMENV_E_INVALID, "base_stock_rollout(NULL)");
  CHECK(imenv_plan_rollout(nullptr, nullptr, nullptr) == IMENV_E_INVALID, "plan_rollout(NULL)");
  CHECK(imenv_set_episode_metrics(nullptr, nullptr) == IMENV_E_INVALID, "set_episode_metrics(NULL)");
  CHECK(imenv_column_stats(nullptr, 4, 2, nullptr, nullptr) == IMENV_E_INVALID, "column_stats(NULL)");
  CHECK(imenv_cc_observation(4, 2, 3, nullptr, IMENV_F32, nullptr, IMENV_F32, -1.0, 1.0, nullptr, nullptr) ==
            IMENV_E_INVALID, "cc_observation(NULL)");
  CHECK(imenv_gae(4, 30, nullptr, IMENV_F64, nullptr, IMENV_F64, nullptr, 0.99, 0.95, nullptr, nullptr, nullptr) ==
            IMENV_E_INVALID, "gae(NULL)");
  CHECK(imenv_set_delay_uniforms(nullptr, 0, nullptr, nullptr) == IMENV_E_INVALID, "set_delay_uniforms(NULL)");
  CHECK(imenv_set_store_policy(nullptr, 0) == IMENV_E_INVALID, "set_store_policy(NULL)");
  CHECK(imenv_set_jit(nullptr, 1) == IMENV_E_INVALID, "set_jit(NULL)");
  int32_t a = 0, b = 0, c = 0, d = 0;
  CHECK(imenv_dims(nullptr, &a, &b, &c, &d) == IMENV_E_INVALID, "dims(NULL)");
  CHECK(imenv_state_layout(nullptr, &a, &b, &c) == IMENV_E_INVALID, "state_layout(NULL)");
  uint32_t tab[4];
  CHECK(imenv_poisson_table(nullptr, tab, 4, &a) == IMENV_E_INVALID, "poisson_table(NULL)");
  char buf[64];
  CHECK(imenv_kernel_info(nullptr, buf, sizeof buf) == IMENV_E_INVALID, "kernel_info(NULL)");
  CHECK(imenv_jit_check(nullptr, "gfx950", 0, buf, sizeof buf) == IMENV_E_INVALID, "jit_check(NULL)");
  imenv_destroy(nullptr);
  CHECK(imenv_last_error() != nullptr && std::strlen(imenv_last_error()) > 0, "last_error after a failure");
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s SPECS.bin\n", argv[0]);
    return 2;
  }
  CHECK(imenv_abi_version() == IMENV_ABI_VERSION, "abi version");
  CHECK(imenv_spec_size() == (int64_t)sizeof(ImEnvSpec), "spec size");
  null_argument_paths();
  FILE* fp = std::fopen(argv[1], "rb");
  if (!fp) {
    std::perror(argv[1]);
    return 2;
  }
  int n_valid = 0, n_rejected = 0, n_jit = 0;
  for (;;) {
    int32_t expect = 0, jit = 0;
    char name[64];
    ImEnvSpec s;
    if (std::fread(&expect, 4, 1, fp) != 1) break;
    if (std::fread(&jit, 4, 1, fp) != 1 || std::fread(name, 64, 1, fp) != 1 || std::fread(&s, sizeof s, 1, fp) != 1) {
      std::fprintf(stderr, "truncated record\n");
      return 2;
    }
    name[63] = 0;
    char log[4096];
    // validation + derivation + obs tables + source generation (+ hipRTC compile for the specs flagged jit)
    const uint32_t flag_sets[] = {0u, 1u | 2u, 2048u, 1024u | (1u << 5)};
    for (uint32_t flags : flag_sets) {
      if (!jit && flags != 0u) break;
      int rc = jit ? imenv_jit_check(&s, "gfx950", flags, log, sizeof log)
                   : imenv_jit_check(&s, "gfx-invalid-arch", flags, log, sizeof log);
      if (expect == 1) {
        CHECK(rejected(rc), "%s: malformed spec accepted by jit_check (rc %d)", name, rc);
        break;
      }
      if (jit) {
        CHECK(rc == IMENV_OK, "%s flags 0x%x: jit_check rc %d: %.300s / %s", name, flags, rc, log, imenv_last_error());
        ++n_jit;
      } else {
        // an unknown arch fails only at the hipRTC compile, after validation and source generation
        CHECK(rc == IMENV_E_UNSUPPORTED && std::strstr(imenv_last_error(), "hipRTC"), "%s: rc %d (%s)", name, rc,
              imenv_last_error());
      }
    }
    ImEnv* h = nullptr;
    int rc = imenv_create(&s, 64, 0, 0, &h);
    if (expect == 1) {
      CHECK(rejected(rc) && h == nullptr, "%s: malformed spec accepted by create (rc %d)", name, rc);
      CHECK(std::strlen(imenv_last_error()) > 0, "%s: no error message", name);
      ++n_rejected;
    } else {
      // no GPU here: create validates, then fails at the first HIP call (or succeeds on a GPU box)
      CHECK(rc == IMENV_OK || rc == IMENV_E_HIP, "%s: create rc %d (%s)", name, rc, imenv_last_error());
      if (h) imenv_destroy(h);
      ++n_valid;
    }
    // out-of-range batch sizes and env offsets
    h = nullptr;
    CHECK(imenv_create(&s, 0, 0, 0, &h) == IMENV_E_INVALID && !h, "%s: n_envs 0", name);
    CHECK(imenv_create(&s, 16, (int64_t(1) << 32) - 8, 0, &h) == IMENV_E_INVALID && !h, "%s: env ids > 32 bits", name);
  }
  std::fclose(fp);
  std::printf("{\"valid_specs\": %d, \"rejected_specs\": %d, \"jit_compiles\": %d, \"failures\": %d}\n", n_valid,
              n_rejected, n_jit, g_fail);
  return g_fail ? 1 : 0;
}
