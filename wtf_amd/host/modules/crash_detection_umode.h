// crash_detection_umode.h — user-mode crash detection breakpoints
// (src/wtf/crash_detection_umode.{h,cc}).
#pragma once
bool SetupUsermodeCrashDetectionHooks();
