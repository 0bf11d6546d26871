// kgmt_sharded.cpp — multi-GPU sharding of one planning problem (placeholder;
// the RCCL exchange lands in the next commit).
#include "kgmt_planner.h"

namespace sbmp {

class Exchange {};

void* sharded_create_comm(const uint8_t*, int, int, int) {
    throw Error(SBMP_ERR_UNSUPPORTED, "sharded planner not built yet");
}
void sharded_destroy_comm(void*) {}
Exchange* sharded_exchange(void*) { return nullptr; }
void comm_get_unique_id(uint8_t*) { throw Error(SBMP_ERR_UNSUPPORTED, "sharded planner not built yet"); }

void KgmtPlanner::enqueue_sharded_iteration(int) {
    throw Error(SBMP_ERR_UNSUPPORTED, "sharded planner not built yet");
}

}  // namespace sbmp
