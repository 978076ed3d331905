// Internal probe hooks (see probe.cpp); kinds mirror CG_PROBE_* in the public header.
#pragma once
#include <hip/hip_runtime.h>

int cg_probe_kind();
void cg_probe_begin(int kind, hipStream_t s);
// work: algorithmic FLOPs of the launch; bytes: its algorithmic HBM bytes (operands once + outputs once)
void cg_probe_end(int kind, hipStream_t s, double work, double bytes = 0.0);
