// TOOLS ONLY: the C entry point of a product parse kernel rebuilt from git history (tools/ab/base/Makefile).
#include "pcppx.h"
#include "pcppx_internal.h"

extern "C" __attribute__((visibility("default"))) int pcppx_r01_parse_device(const pcppx_batch* b, const pcppx_opts* o,
                                                                             pcppx_records* r, void* stream)
{
	return pcppx::launch_parse(b, o, r, static_cast<hipStream_t>(stream));
}
