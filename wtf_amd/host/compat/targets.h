// compat/targets.h — the reference header of the same name (src/wtf/targets.h), for
// building an upstream module source unchanged against this backend: the
// declarations it needs are in wtf_api.h (see compat/README.md).
#pragma once
#include "../wtf_api.h"
