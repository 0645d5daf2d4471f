// wavefront_primary.hip -- the wavefront's bounce-0 packet extend
// (wavefront.hip wf_extend_primary) in a translation unit of its own.
//
// Its walk is driven by wave-uniform decisions (ballots over the lanes of one
// 8x8 primary-ray tile), and it is compiled with the uniform regions of its
// control flow left unstructurized (_build.py: -structurizecfg-skip-uniform-
// regions): plain scalar branches instead of exec-mask bookkeeping, -9% of its
// time (C2 +1.6%).  The same flag on the whole of wavefront.hip slows the
// shade (+5% on C2, +9% on C4: C4 -3%), hence the split.
#define MCPT_WF_PRIMARY_TU 1
#include "wavefront.hip"
