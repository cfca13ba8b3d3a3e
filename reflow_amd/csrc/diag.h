// diag.h -- A/B and diagnostic switches (measured-dead kernel forms,
// wrong-digest timing probes, phase stamps, host-leg tuning probes): read from
// the environment only by a diagnostic build (-DRF_DIAG, e.g. make
// EXTRA=-DRF_DIAG BUILD=build_diag OUT=../../tools/_diag/libreflow_hip.so);
// the product library compiles to the defaults, and neither the names nor the
// code paths they select are in it.  Internal, host code only.
#pragma once
#ifdef RF_DIAG
#include <cstdlib>
#define RF_DIAG_KNOB(name, dflt) (getenv(name) ? strtol(getenv(name), nullptr, 10) : (long)(dflt))
#else
#define RF_DIAG_KNOB(name, dflt) ((long)(dflt))
#endif
