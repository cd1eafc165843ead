// compat/pch.h — the reference's precompiled header (src/wtf/pch.h), which its
// build forces into every translation unit (src/CMakeLists.txt:137-141): module
// sources rely on names it brings in (the `json` alias, span_u8, _1MB, ...).
// Here it pulls the compat headers; pass it with -include as upstream does.
#pragma once
#include "backend.h"
#include "corpus.h"
#include "debugger.h"
#include "globals.h"
#include "mutator.h"
#include "targets.h"
#include "utils.h"
