// bqp_ocp_f32.hip — fp32 instantiation of the structured kernel (bqp_ocp.hip): the same source
// with `real` = float for the solver's LDS state and arithmetic (config C5, "fp32 vs fp64").
// The caller's arrays stay fp64 in HBM.  Entry points: launch_ocp_f32, ocp_wave_lds_doubles_f32.
#define BQP_F32 1
#include "bqp_ocp.hip"
