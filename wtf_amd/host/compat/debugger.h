// compat/debugger.h — the reference header of the same name (src/wtf/debugger.h),
// for building an upstream module source unchanged against this backend:
// Debugger_t / g_Dbg are in wtf_api.h; the header also brings the `json`
// namespace alias the reference modules use (debugger.h:15) when nlohmann/json
// is on the include path, as it is in the upstream tree.
#pragma once
#include "../wtf_api.h"
#if __has_include(<nlohmann/json.hpp>)
#include <nlohmann/json.hpp>
namespace json = nlohmann;
#endif
