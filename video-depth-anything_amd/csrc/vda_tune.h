// Route and schedule knobs.  The product library (`make` -> libvda.so) keeps no mutable global state:
// every knob below is a compile-time constant at its automatic value, and the vda_debug_* entry points
// do not exist.  The tuning build (`make tune` -> build/tune/libvda.so, -DVDA_TUNING) turns the knobs
// into process-global variables set through the entry points of include/vda_tune.h, for A/B runs and
// for the tests that compare the alternative kernel routes with the default one.
#pragma once
#ifdef VDA_TUNING
#define VDA_KNOB(type, name, value) type name = value
#else
#define VDA_KNOB(type, name, value) constexpr type name = value
#endif
