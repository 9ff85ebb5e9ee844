// cfx_internal.h — library-internal accessors shared between the translation units of libcfx (not part of the
// C ABI in include/cfx.h).
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "../../include/cfx.h"

// last failure of a handle-free call on this thread (cfx_last_error(NULL))
extern thread_local std::string g_create_error;

// batch, layout, device and launch stream of a handle (cfx_api.hip)
int cfx_internal_info(const cfx_handle* h, int64_t* batch, int* layout, int* device, hipStream_t* stream);
