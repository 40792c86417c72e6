// hd_tally.hip -- placeholder; the GPU tally lands in the next commit.
#include "hd_internal.h"
void hd_tally_release(hd_ctx*) {}
extern "C" {
int hd_tally(hd_ctx*, const hd_batch*, const uint8_t*, hd_tally_out*) { return HD_EINVAL; }
int hd_process_batch(hd_ctx*, const hd_batch*, uint8_t*, uint8_t*, uint32_t*, hd_tally_out*) { return HD_EINVAL; }
}
