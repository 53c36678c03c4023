// One group of kernels of liblodestar_bls.so, compiled once per group with -DLB_KGROUP=g
// (tools/gen_kdecls.py GROUPS); lb_engine.hip launches them through lb_kdecl.h.
#define LB_KDECL_INSTANTIATE
#include "lb_kernels.h"
#include "lb_kzg.h"
#include "lb_kdecl.h"
