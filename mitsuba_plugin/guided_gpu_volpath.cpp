// src/integrators/path/guided_gpu_volpath.cpp -- the volumetric plugin: SD-tree guided progressive
// volumetric path tracer on the MI355X (ProgressiveVolumetricPathTracer's surface,
// progressive_volpath.cpp:71-470: homogeneous and heterogeneous media flattened to pg_medium, HG phase,
// null-BSDF medium transitions; guided distance sampling with `distanceGuiding`), over the pg C-ABI.
#include "guided_gpu.h"

MTS_NAMESPACE_BEGIN

class GuidedGPUVolPathTracer : public GuidedGPUIntegrator {
public:
    GuidedGPUVolPathTracer(const Properties &props) : GuidedGPUIntegrator(props, true) { }
    GuidedGPUVolPathTracer(Stream *s, InstanceManager *m) : GuidedGPUIntegrator(s, m) { }
    MTS_DECLARE_CLASS()
};

MTS_IMPLEMENT_CLASS_S(GuidedGPUVolPathTracer, false, ProgressiveMonteCarloIntegrator)
MTS_EXPORT_PLUGIN(GuidedGPUVolPathTracer, "Guided progressive volumetric path tracer (MI355X)");
MTS_NAMESPACE_END
