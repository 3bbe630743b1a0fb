// tpt_conn2.hip -- the walk-group scenes' connect kernel (tpt_bdpt_conn_kernel<2>, defined
// in tpt_capi.hip) in a translation unit of its own, so that it can be built without the
// AMDGPU register-pressure trackers (Makefile): with them this compiler segfaults in its
// machine scheduler on that kernel for some code shapes.  tpt_capi.hip declares the
// instantiation `extern template` and launches it; nothing else is compiled here.
#define TPT_TU_CONN2 1
#include "tpt_capi.hip"

template __global__ void tpt_bdpt_conn_kernel<2, TPT_CONN_QUEUE_WALK != 0>(DScene, WfState, float*);
