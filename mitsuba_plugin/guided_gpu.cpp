// src/integrators/path/guided_gpu.cpp -- the surface plugin: SD-tree guided progressive path tracer
// on the MI355X (ProgressiveMIPathTracer's surface, progressive_path.cpp:89-341), over the pg C-ABI.
#include "guided_gpu.h"

MTS_NAMESPACE_BEGIN

class GuidedGPUPathTracer : public GuidedGPUIntegrator {
public:
    GuidedGPUPathTracer(const Properties &props) : GuidedGPUIntegrator(props, false) { }
    GuidedGPUPathTracer(Stream *s, InstanceManager *m) : GuidedGPUIntegrator(s, m) { }
    MTS_DECLARE_CLASS()
};

MTS_IMPLEMENT_CLASS_S(GuidedGPUPathTracer, false, ProgressiveMonteCarloIntegrator)
MTS_EXPORT_PLUGIN(GuidedGPUPathTracer, "Guided progressive path tracer (MI355X)");
MTS_NAMESPACE_END
