// pgmg_comm.hip — row-strip domain decomposition over RCCL (one process per GPU).
// (placeholder until the strip exchange lands; world == 1 never reaches here)
#include "pgmg_ctx.h"

namespace pgmg {

Comm *Comm::create(pgmg_ctx *c, int *rc)
{
    (void)c;
    *rc = set_err(PGMG_ERR_STATE, "world > 1 not available in this build");
    return nullptr;
}

}  // namespace pgmg

extern "C" int pgmg_comm_unique_id(void *out128)
{
    (void)out128;
    return pgmg::set_err(PGMG_ERR_STATE, "RCCL bootstrap not available in this build");
}
