// halo.cpp -- processor-patch halo exchange over RCCL (replaces dfNcclBase.cu:23-65 and
// correct_boundary_conditions_processor_*, dfMatrixOpBase.cu:441-485, 1366-1389).
#include "dfmi_ctx.h"

namespace dfmi {
struct Halo {};
void halo_destroy(Halo* h) { delete h; }
Ctx::~Ctx() { halo_destroy(halo); }
void halo_exchange(Ctx& x, double*, int, long) {
  for (int k : x.pkind) DFMI_CHECK(k != 2, "processor patches need dfmi_set_comm_info (RCCL halo)");
}
}  // namespace dfmi
