// TOOLS ONLY: the C entry point of the round-1 parse kernel (built from git history by tools/ab/r01/Makefile).
#include "pcppx.h"
#include "pcppx_internal.h"

extern "C" __attribute__((visibility("default"))) int pcppx_r01_parse_device(const pcppx_batch* b, const pcppx_opts* o,
                                                                             pcppx_records* r, void* stream)
{
	return pcppx::launch_parse(b, o, r, static_cast<hipStream_t>(stream));
}
