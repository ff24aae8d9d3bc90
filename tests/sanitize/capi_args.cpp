// Host-side ASan / UBSan exercise of the C ABI's argument validation (sanitizers
// on the host runtime).  Built by `make -C pnp-pds_amd sanitize` with -fsanitize=address,undefined
// on the host side of every translation unit (device code unchanged), run by
// tests/test_sanitize.py on the CPU box: no GPU is needed, every call here fails before a launch
// or is host-only.  Exit status 0 = every expectation held and no sanitizer report.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/pnppds.h"

static int failures = 0;
#define EXPECT(cond)                                                       \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "%s:%d: expected %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

int main() {
  EXPECT(pnp_abi_version() == PNP_ABI_VERSION);
  EXPECT(std::strlen(pnp_build_id()) == 16);
  EXPECT(pnp_device_count(nullptr) == PNP_E_ARG);
  int n = -1;
  const int rc = pnp_device_count(&n);
  EXPECT(rc == PNP_OK || rc == PNP_E_HIP);
  EXPECT(pnp_create(0, nullptr) == PNP_E_ARG);
  pnp_ctx* ctx = reinterpret_cast<pnp_ctx*>(0x1);
  const int rc_create = pnp_create(0, &ctx);
  if (rc_create != PNP_OK) {                      // no device here: the error path, ctx cleared
    EXPECT(ctx == nullptr);
    EXPECT(std::strlen(pnp_last_error(nullptr)) > 0);
  } else {
    pnp_destroy(ctx);
  }
  EXPECT(pnp_create(-1, &ctx) != PNP_OK);
  EXPECT(pnp_destroy(nullptr) == PNP_OK);

  // every entry point rejects a NULL context
  pnp_params prm{};
  float f = 0.f;
  double d = 0.0;
  int k = 0;
  const float* cp = nullptr;
  const char* name = nullptr;
  EXPECT(pnp_synchronize(nullptr) == PNP_E_ARG);
  EXPECT(pnp_set_denoiser(nullptr, 3, 20, 64, &f, 1, 0, 1, 1) == PNP_E_ARG);
  EXPECT(pnp_set_precision(nullptr, PNP_PREC_AUTO) == PNP_E_ARG);
  EXPECT(pnp_get_precision(nullptr, &k, &k) == PNP_E_ARG);
  EXPECT(pnp_set_precision(nullptr, PNP_PREC_CONVERGE) == PNP_E_ARG);
  EXPECT(pnp_get_precision_switch(nullptr, &k) == PNP_E_ARG);
  EXPECT(pnp_get_precision_switches(nullptr, &k, 1) == PNP_E_ARG);
  EXPECT(pnp_set_tuning(nullptr, 0, 0) == PNP_E_ARG);
  EXPECT(pnp_set_operator(nullptr, PNP_OP_ID, nullptr, 0, 0, nullptr, 0, 0) == PNP_E_ARG);
  EXPECT(pnp_run(nullptr, PNP_METHOD_A, &prm, 1, 3, 8, 8, &f, &f, &f, 1, &f, &f, &d, &d, &d, &d) == PNP_E_ARG);
  EXPECT(pnp_solver_setup(nullptr, PNP_METHOD_A, &prm, 1, 3, 8, 8, 1) == PNP_E_ARG);
  EXPECT(pnp_solver_load(nullptr, &f, &f, &f) == PNP_E_ARG);
  EXPECT(pnp_solver_load_device(nullptr, &f, &f, &f) == PNP_E_ARG);
  EXPECT(pnp_solver_iterate(nullptr, 1) == PNP_E_ARG);
  EXPECT(pnp_solver_fetch(nullptr, &f, &f, &d, &d, &d) == PNP_E_ARG);
  EXPECT(pnp_solver_iterations_done(nullptr, &k) == PNP_E_ARG);
  EXPECT(pnp_solver_state(nullptr, &cp, &cp, &cp) == PNP_E_ARG);
  EXPECT(pnp_profile_enable(nullptr, 1) == PNP_E_ARG);
  EXPECT(pnp_profile_read(nullptr, 1, &name, &d, &k, &k) == PNP_E_ARG);
  EXPECT(pnp_op_phi(nullptr, &f, &f, 1, 1, 1, 1, nullptr) == PNP_E_ARG);
  EXPECT(pnp_op_adj_phi(nullptr, &f, &f, 1, 1, 1, 1, nullptr) == PNP_E_ARG);
  EXPECT(pnp_op_proj_l2_ball(nullptr, &f, &f, &f, 1, 1, 1, 1, 0, 1, nullptr) == PNP_E_ARG);
  EXPECT(pnp_op_proj_l1_ball(nullptr, &f, &f, 1, 1, 1, 0.1, 1, nullptr) == PNP_E_ARG);
  EXPECT(pnp_op_prox_gkl(nullptr, &f, &f, &f, 1, 1, 1, nullptr) == PNP_E_ARG);
  EXPECT(pnp_op_denoise(nullptr, &f, &f, 1, 3, 8, 8, nullptr) == PNP_E_ARG);
  EXPECT(pnp_op_status(nullptr, nullptr) == PNP_E_ARG);
  EXPECT(pnp_device_copy(nullptr, &f, &f, 16, nullptr) == PNP_E_ARG);
  EXPECT(pnp_op_psnr(nullptr, &f, &f, 1, 1, &d, nullptr) == PNP_E_ARG);
  EXPECT(pnp_op_ssim(nullptr, &f, &f, 1, 1, 8, 8, &d, nullptr) == PNP_E_ARG);
  pnp_degrade_params dp{};
  EXPECT(pnp_degrade(nullptr, &dp, 1, 3, 8, 8, &f, &f, &f, &d, nullptr) == PNP_E_ARG);

  // the host-only weight rounding: bounds, aliasing, edge values
  EXPECT(pnp_fp16_filter_round(nullptr, 1, &f) == PNP_E_ARG);
  EXPECT(pnp_fp16_filter_round(&f, 1, nullptr) == PNP_E_ARG);
  std::mt19937 rng(7);
  std::normal_distribution<float> nd(0.f, 0.05f);
  std::vector<float> w(9 * 4096), out(w.size());
  for (auto& v : w) v = nd(rng);
  for (int i = 0; i < 9; ++i) w[i] = 0.f;                        // an all-zero filter
  for (int i = 9; i < 18; ++i) w[i] = 6e-8f * (float)(i - 13);   // fp16 subnormals
  EXPECT(pnp_fp16_filter_round(w.data(), w.size() / 9, out.data()) == PNP_OK);
  for (size_t i = 0; i < w.size(); ++i) {
    EXPECT(std::isfinite(out[i]));
    EXPECT((float)(_Float16)out[i] == out[i]);
    if (failures > 20) break;
  }
  std::vector<float> alias = w;
  EXPECT(pnp_fp16_filter_round(alias.data(), alias.size() / 9, alias.data()) == PNP_OK);
  EXPECT(std::memcmp(alias.data(), out.data(), out.size() * 4) == 0);
  EXPECT(pnp_fp16_filter_round(w.data(), 0, out.data()) == PNP_OK);

  if (failures) std::fprintf(stderr, "%d failures\n", failures);
  else std::printf("capi_args ok\n");
  return failures ? 1 : 0;
}
