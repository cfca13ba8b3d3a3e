// errors.cpp -- rf_last_error() / rf_version() and rf::fail (host-only).
#include <cstdarg>
#include <cstdio>
#include <string>

#include "errors.h"

// ---------------------------------------------------------------------------
// errors (errors.h)
static thread_local std::string g_err;

int rf::fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

extern "C" const char* rf_last_error(void) { return g_err.c_str(); }
extern "C" const char* rf_version(void) { return "reflow-hip 0.2 gfx950"; }

