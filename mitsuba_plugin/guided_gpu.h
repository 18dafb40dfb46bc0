// Mitsuba plugin adapter over the pg C-ABI (include/pg_capi.h): the drop-in boundary of SURVEY.md §8b.
//
// A maintainer copies mitsuba_plugin/ into the fork's src/integrators/path/ and adds two plugins
// (INTEGRATION.md has the CMake lines):
//   guided_gpu          GuidedGPUPathTracer     -> ProgressiveMIPathTracer's surface   (progressive_path.cpp:89-341)
//   guided_gpu_volpath  GuidedGPUVolPathTracer  -> ProgressiveVolumetricPathTracer's  (progressive_volpath.cpp:71-470)
// Both are ProgressiveMonteCarloIntegrators (progressiveintegrator.h:10-86): preprocess flattens the
// scene (TriMesh arrays, BSDF parameters, area emitters, the environment emitter, participating
// media, camera) into a pg_scene_desc and uploads it; render runs the training progressions (render
// pass with records, postprogression exchange + refit) and the final progressions through the C-ABI
// and writes the film; Li() keeps renderBlock()/E() working through Mitsuba's own CPU integrator.
//
// This file cannot be compiled in the repository's container: it needs the fork's headers and their
// Boost / Xerces / OpenEXR / OIDN dependencies.  integrator.py makes the same C-ABI
// calls in the same order and is what the tests run.
#pragma once
#include <mitsuba/render/progressiveintegrator.h>
#include <mitsuba/render/scene.h>
#include <mitsuba/render/trimesh.h>
#include <mitsuba/render/medium.h>
#include <mitsuba/render/phase.h>
#include <mitsuba/render/sensor.h>
#include <mitsuba/render/ior.h>
#include <mitsuba/core/bitmap.h>
#include <mitsuba/core/plugin.h>
#include <mitsuba/core/fresolver.h>
#include <mitsuba/core/fstream.h>
#include <mitsuba/core/timer.h>
#include <mitsuba/render/denoiser.h>
#include <boost/algorithm/string.hpp>
#include <map>
#include <thread>
#include <pg_capi.h>

MTS_NAMESPACE_BEGIN

class GuidedGPUIntegrator : public ProgressiveMonteCarloIntegrator {
public:
    GuidedGPUIntegrator(const Properties &props, bool volumetric) : ProgressiveMonteCarloIntegrator(props) {
        pg_config_default(&m_cfg);
        m_cfg.integrator = volumetric ? PG_INTEGRATOR_VOLPATH : PG_INTEGRATOR_PATH;
        m_cfg.max_depth = m_maxDepth;                       // MonteCarloIntegrator (integrator.cpp:195-230)
        m_cfg.rr_depth = m_rrDepth;
        m_cfg.strict_normals = m_strictNormals;
        m_cfg.hide_emitters = m_hideEmitters;
        m_cfg.use_nee = props.getBoolean("useNee", true);   // progressive_path.cpp:117
        m_cfg.max_component_value = m_maxComponentValue;   // progressiveintegrator.cpp:296-300
        m_cfg.guiding = props.getBoolean("guiding", true);
        m_cfg.bsdf_sampling_fraction = props.getFloat("bsdfSamplingFraction", 0.5f);
        m_cfg.s_tree_threshold = props.getFloat("sTreeThreshold", 12000.f);
        m_cfg.d_tree_threshold = props.getFloat("dTreeThreshold", 0.01f);
        m_cfg.distance_guiding = props.getFloat("distanceGuiding", m_cfg.distance_guiding);  // volpath only
        // denoiser feature buffers (the fork's OIDN wrapper, denoiser.h): the first hit's BSDF::getAlbedo
        // and shading normal per camera sample, averaged per pixel on the device; after the render the
        // adapter feeds the means to Denoiser and stores its buffers ("denoiserFile"); with
        // denoise = true the film receives the denoised image
        m_cfg.aovs = props.getBoolean("aovs", false);
        m_denoise = props.getBoolean("denoise", false);
        m_denoiserFile = props.getString("denoiserFile", "");
        if (volumetric && (m_cfg.aovs || m_denoise || !m_denoiserFile.empty()))  // pg_create: aovs need the path integrator
            Log(EError, "guided_gpu_volpath: \"aovs\", \"denoise\" and \"denoiserFile\" are supported by guided_gpu only");
        if (m_denoise || !m_denoiserFile.empty()) m_cfg.aovs = 1;
        // combination of the training iterations' images with the final render: "discard" (Mueller et al.
        // 2017's default: the final render only) or "inversevar" (each image weighted by the inverse of
        // its mean per-pixel variance; integrator.py combine_inverse_variance is the same arithmetic)
        m_sampleCombination = boost::to_lower_copy(props.getString("sampleCombination", "discard"));
        if (m_sampleCombination != "discard" && m_sampleCombination != "inversevar")
            Log(EError, "guided_gpu: sampleCombination must be \"discard\" or \"inversevar\"");
        // volpath: MIS of emitters behind index-matched surfaces with the whole ray length (unbiased)
        // instead of the reference's last segment
        m_cfg.volpath_exact_mis = props.getBoolean("exactMis", false);
        // a chunk with at most this many live paths finishes in one launch (k_tail); 0 = library default
        m_cfg.tail_paths = props.getInteger("tailPaths", 0);
        // BSDF::getGlossySamplingRate as a prior on the BSDF fraction (glossy lobes are not guided)
        m_cfg.glossy_prior = props.getBoolean("glossyPrior", m_cfg.glossy_prior != 0);
        std::string bound = boost::to_lower_copy(props.getString("bsdfSamplingFractionBound", "fixed"));
        m_cfg.bsdf_fraction_bound = bound == "albedo" ? PG_FRACTION_ALBEDO : bound == "learned" ? PG_FRACTION_LEARNED
                                    : bound == "throughput" ? PG_FRACTION_THROUGHPUT : PG_FRACTION_FIXED;
        // multi-GPU: one Mitsuba process per GPU (e.g. mitsuba -Drank=2 -DworldSize=8 scene.xml); the
        // context renders its 32x32 tile shard, rank 0 writes the whole image
        m_cfg.rank = props.getInteger("rank", 0);
        m_cfg.world_size = props.getInteger("worldSize", 1);
        m_cfg.device = props.getInteger("device", m_cfg.rank);
        m_commIdFile = props.getString("commIdFile", "guided_gpu.commid");
        // postprogression exchange between ranks: "allreduce" (the building statistics, a few MB) or
        // "allgather" (every rank's training records, SURVEY.md §5: the record all-gather) -- the same tree
        m_exchange = boost::to_lower_copy(props.getString("exchange", "allreduce"));
        if (m_exchange != "allreduce" && m_exchange != "allgather")
            Log(EError, "guided_gpu: exchange must be \"allreduce\" or \"allgather\"");
        m_trainingIterations = props.getInteger("trainingIterations", 5);
        m_maxRenderTime = props.getFloat("maxRenderTime", 0.0f);  // progressiveintegrator.cpp:117-168
        m_mediumResolution = props.getInteger("mediumResolution", 256);  // heterogeneous media, per axis
    }
    GuidedGPUIntegrator(Stream *s, InstanceManager *m) : ProgressiveMonteCarloIntegrator(s, m) {
        s->read(&m_cfg, sizeof(m_cfg));
        m_trainingIterations = s->readInt();
        m_maxRenderTime = s->readFloat();
        m_commIdFile = s->readString();
        m_exchange = s->readString();
        m_mediumResolution = s->readInt();
        m_sampleCombination = s->readString();
        m_denoiserFile = s->readString();
        m_denoise = s->readBool();
    }
    void serialize(Stream *s, InstanceManager *m) const override {
        ProgressiveMonteCarloIntegrator::serialize(s, m);
        s->write(&m_cfg, sizeof(m_cfg));
        s->writeInt(m_trainingIterations);
        s->writeFloat(m_maxRenderTime);
        s->writeString(m_commIdFile);
        s->writeString(m_exchange);
        s->writeInt(m_mediumResolution);
        s->writeString(m_sampleCombination);
        s->writeString(m_denoiserFile);
        s->writeBool(m_denoise);
    }

    bool preprocess(const Scene *scene, RenderQueue *queue, const RenderJob *job,
                    int sceneResID, int sensorResID, int samplerResID) override {
        ProgressiveMonteCarloIntegrator::preprocess(scene, queue, job, sceneResID, sensorResID, samplerResID);
        check(pg_create(&m_cfg, &m_ctx));
        m_flat = flatten(scene);  // TriMesh arrays, BSDFs, emitters (area + environment), media, camera
        m_flat.bind();            // the descriptor's pointers into this copy's arrays
        check(pg_upload_scene(m_ctx, &m_flat.desc));
        if (m_cfg.world_size > 1) initComm();
        // Li() / renderBlock() / E() keep working through Mitsuba's own CPU integrator (not guided)
        Properties pp(m_cfg.integrator == PG_INTEGRATOR_VOLPATH ? "volpath" : "path");
        pp.setInteger("maxDepth", m_maxDepth);
        pp.setInteger("rrDepth", m_rrDepth);
        pp.setBoolean("strictNormals", m_strictNormals);
        pp.setBoolean("hideEmitters", m_hideEmitters);
        m_cpu = static_cast<SamplingIntegrator *>(PluginManager::getInstance()->
                    createObject(MTS_CLASS(SamplingIntegrator), pp));
        m_cpu->configure();
        return true;
    }

    bool render(Scene *scene, RenderQueue *queue, const RenderJob *job,
                int sceneResID, int sensorResID, int samplerResID) override {
        ref<Timer> timer = new Timer();
        uint32_t offset = 0;
        const size_t npix = (size_t) m_flat.desc.camera.width * m_flat.desc.camera.height;
        m_iterationFilms.clear();
        for (int it = 0; it < m_trainingIterations && m_cfg.guiding; ++it) {   // training progressions
            preprogression(queue, job, sceneResID, sensorResID, samplerResID);
            if (!pass(1u << it, offset, 1)) return false;
            offset += 1u << it;
            if (m_sampleCombination == "inversevar") {           // keep this iteration's image (this rank's tiles)
                FilmSums f;
                f.rgbw.resize(4 * npix);
                f.sumsq.resize(4 * npix);
                check(pg_read_film(m_ctx, f.rgbw.data(), f.sumsq.data()));
                check(pg_reset_film(m_ctx));
                m_iterationFilms.push_back(std::move(f));
            }
            if (m_cfg.world_size > 1 && m_exchange == "allgather") {
                check(pg_comm_allgather_records(m_ctx, NULL));  // RCCL: every rank splats every rank's records
            } else {
                check(pg_splat_local_records(m_ctx));            // this rank's records -> building tree
                if (m_cfg.world_size > 1)
                    check(pg_comm_allreduce_tree_stats(m_ctx));  // RCCL: sum of every rank's statistics
            }
            check(pg_refit(m_ctx, it));                          // the postprogression refit slot
            postprogression(queue, job, sceneResID, sensorResID, samplerResID);
        }
        check(pg_reset_film(m_ctx));
        if (m_maxRenderTime > 0 && m_cfg.world_size > 1) {
            // renderTime with a tile shard: every rank must render the same whole progressions, so each
            // batch is sized from all-reduced clocks (the slowest rank's elapsed time and seconds per
            // progression; integrator.py _render_time_sharded does the same over torch.distributed)
            const int W = m_cfg.world_size;
            uint32_t done = 0;
            double perProg = 0;
            for (;;) {
                std::vector<double> v(2 * W, 0.0);
                v[m_cfg.rank] = timer->getMilliseconds() * 1e-3;
                v[W + m_cfg.rank] = perProg;
                check(pg_comm_allreduce_f64(m_ctx, v.data(), v.size()));
                const double el = *std::max_element(v.begin(), v.begin() + W);
                const double pp = *std::max_element(v.begin() + W, v.end());
                if (el >= m_maxRenderTime) break;
                const uint32_t progs = done == 0 ? 1u : (uint32_t) std::max(1.0, std::min(
                    std::floor(0.5 * (m_maxRenderTime - el) / std::max(pp, 1e-9)), 1e6));
                const double t0 = timer->getMilliseconds() * 1e-3;
                preprogression(queue, job, sceneResID, sensorResID, samplerResID);
                if (!pass(progs * m_samplesPerProgression, offset + done, 0)) return false;
                postprogression(queue, job, sceneResID, sensorResID, samplerResID);
                done += progs * m_samplesPerProgression;
                perProg = (timer->getMilliseconds() * 1e-3 - t0) / progs;
            }
            m_spp = done;
        } else if (m_maxRenderTime > 0) {                        // renderTime (progressiveintegrator.cpp:117-168)
            const double left = m_maxRenderTime - timer->getMilliseconds() * 1e-3;
            uint32_t done = 0;
            pg_status st = left > 0 ? pg_render_time(m_ctx, left, m_samplesPerProgression, offset, 0, &done) : PG_OK;
            if (st == PG_ERR_CANCELLED) return false;
            check(st);
            m_spp = done;                                        // what renderTime reports
        } else {
            for (int done = 0; done < m_spp; done += m_samplesPerProgression) {
                preprogression(queue, job, sceneResID, sensorResID, samplerResID);
                if (!pass(m_samplesPerProgression, offset, 0)) return false;
                offset += m_samplesPerProgression;
                postprogression(queue, job, sceneResID, sensorResID, samplerResID);
            }
        }
        // the image: per pixel (sum rgb, count); the film sums of this rank's tiles
        std::vector<float> rgbw(4 * npix);
        if (m_sampleCombination == "inversevar" && !m_iterationFilms.empty()) {
            FilmSums last;
            last.rgbw.resize(4 * npix);
            last.sumsq.resize(4 * npix);
            check(pg_read_film(m_ctx, last.rgbw.data(), last.sumsq.data()));
            m_iterationFilms.push_back(std::move(last));
            combineInverseVariance(rgbw);                        // weights agree over ranks (all-reduced)
            if (m_cfg.world_size > 1) {                          // disjoint tiles: the sum over ranks is the image
                std::vector<double> img(rgbw.begin(), rgbw.end());
                check(pg_comm_allreduce_f64(m_ctx, img.data(), img.size()));
                for (size_t i = 0; i < img.size(); ++i) rgbw[i] = (float) img[i];
            }
        }
        if (m_cfg.world_size > 1) {
            check(pg_comm_reduce_film(m_ctx, 0));                // RCCL: disjoint tiles (and features) on rank 0
            if (m_cfg.rank != 0) return true;                    // only rank 0 develops the film
        }
        if (m_sampleCombination != "inversevar" || m_iterationFilms.empty())
            check(pg_read_film(m_ctx, rgbw.data(), NULL));
        Film *film = scene->getSensor()->getFilm();
        Vector2i size = film->getSize();
        // the film read-out index of output pixel (x, y): a mirrored toWorld flips x
        auto src = [&](int x, int y) { return (size_t) y * size.x + (m_flat.mirrorX ? size.x - 1 - x : x); };
        std::unique_ptr<Denoiser> denoiser;
        // the OIDN filter runs only when its output is wanted (the film or the stored buffers); "aovs"
        // alone keeps the feature buffers on the context (pg_read_aovs)
        if (m_cfg.aovs && (m_denoise || !m_denoiserFile.empty())) {  // Denoiser::add's inputs (denoiser.cpp:138-144)
            std::vector<float> alb(4 * npix), nrm(4 * npix);
            check(pg_read_aovs(m_ctx, alb.data(), nrm.data()));
            denoiser.reset(new Denoiser());
            denoiser->init(size, true);
            for (int y = 0; y < size.y; ++y)
                for (int x = 0; x < size.x; ++x) {
                    const size_t i = src(x, y);
                    const float w = std::max(rgbw[4 * i + 3], 1.0f), n = std::max(alb[4 * i + 3], 1.0f);
                    Denoiser::Sample smp;                         // one add of the pixel means = their average
                    smp.color.fromLinearRGB(rgbw[4 * i] / w, rgbw[4 * i + 1] / w, rgbw[4 * i + 2] / w);
                    smp.albedo.fromLinearRGB(alb[4 * i] / n, alb[4 * i + 1] / n, alb[4 * i + 2] / n);
                    smp.normal = Vector3(nrm[4 * i] / n, nrm[4 * i + 1] / n, nrm[4 * i + 2] / n);
                    if (m_flat.mirrorX) smp.normal.x = -smp.normal.x;  // the image's x axis is flipped
                    denoiser->add(y * size.x + x, smp);
                }
            denoiser->denoise();
            if (!m_denoiserFile.empty()) denoiser->storeBuffers(m_denoiserFile);
        }
        ref<ImageBlock> block = new ImageBlock(Bitmap::ESpectrumAlphaWeight, size, NULL);
        for (int y = 0; y < size.y; ++y)
            for (int x = 0; x < size.x; ++x) {
                Spectrum s;
                if (m_denoise) {
                    s = denoiser->get(y * size.x + x);
                } else {
                    const float *p = &rgbw[4 * src(x, y)];
                    Float w = std::max(p[3], 1.0f);
                    s.fromLinearRGB(p[0] / w, p[1] / w, p[2] / w);
                }
                block->getBitmap()->setPixel(Point2i(x, y), s);  // box filter: one value per pixel
            }
        film->setBitmap(block->getBitmap());
        return true;
    }

    void cancel() override { if (m_ctx) pg_cancel(m_ctx); ProgressiveMonteCarloIntegrator::cancel(); }

    void postprocess(const Scene *, RenderQueue *, const RenderJob *, int, int, int) override {
        pg_stats st;
        if (m_ctx && pg_get_stats(m_ctx, &st) == PG_OK)
            Log(EInfo, "GPU: %llu paths, %.2f segments/path", (unsigned long long) st.paths,
                st.paths ? (double) st.segments / st.paths : 0.0);
        pg_destroy(m_ctx);                                       // also destroys the RCCL communicator
        m_ctx = NULL;
    }

    // renderBlock() and E() callers get Mitsuba's own (unguided) CPU integrator, same parameters
    Spectrum Li(const RayDifferential &r, RadianceQueryRecord &rRec) const override { return m_cpu->Li(r, rRec); }

protected:
    // every pg_status is checked: Log(EError, ...) throws (formatter.h:33) and ends the job
    void check(pg_status s) const { if (s != PG_OK) Log(EError, "guided_gpu: %s", pg_last_error(m_ctx)); }
    bool pass(uint32_t spp, uint32_t offset, int32_t record) {
        pg_status st = pg_render_pass(m_ctx, spp, offset, record);
        if (st == PG_ERR_CANCELLED) return false;
        check(st);
        return true;
    }
    // Inverse-variance combination of m_iterationFilms (training iterations + the final render): image
    // i has per-pixel means m_i and the variance estimate v_i = the mean over rendered pixels and
    // channels of (E[x^2] - m_i^2) / n; weights 1 / v_i (normalised; the sums are all-reduced over
    // ranks so every tile shard uses the same weights).  out: per pixel (combined mean x total count,
    // total count), i.e. film sums.  integrator.py combine_inverse_variance is the same arithmetic.
    void combineInverseVariance(std::vector<float> &out) const {
        const size_t K = m_iterationFilms.size(), npix = out.size() / 4;
        std::vector<double> st(2 * K, 0.0);
        for (size_t k = 0; k < K; ++k) {
            const FilmSums &f = m_iterationFilms[k];
            for (size_t i = 0; i < npix; ++i) {
                const float cnt = f.rgbw[4 * i + 3];
                if (!(cnt > 0)) continue;
                for (int c = 0; c < 3; ++c) {
                    const float m = f.rgbw[4 * i + c] / cnt, m2 = f.sumsq[4 * i + c] / cnt;
                    st[2 * k] += (double) (std::max(m2 - m * m, 0.0f) / cnt);
                    st[2 * k + 1] += 1.0;
                }
            }
        }
        if (m_cfg.world_size > 1) check(pg_comm_allreduce_f64(m_ctx, st.data(), st.size()));
        std::vector<double> w(K, 0.0);
        double wsum = 0;
        for (size_t k = 0; k < K; ++k) {
            const double v = st[2 * k + 1] > 0 ? st[2 * k] / st[2 * k + 1] : 0.0;
            w[k] = v > 0 && std::isfinite(v) ? 1.0 / v : 0.0;
            wsum += w[k];
        }
        if (!(wsum > 0)) {                                       // no variance estimate: the final render
            std::fill(w.begin(), w.end(), 0.0);
            w[K - 1] = wsum = 1.0;
        }
        for (size_t i = 0; i < npix; ++i) {
            double total = 0, mean[3] = {0, 0, 0};
            for (size_t k = 0; k < K; ++k) {
                const FilmSums &f = m_iterationFilms[k];
                const float cnt = f.rgbw[4 * i + 3], n = std::max(cnt, 1.0f);
                total += cnt;
                for (int c = 0; c < 3; ++c) mean[c] += w[k] / wsum * (f.rgbw[4 * i + c] / n);
            }
            for (int c = 0; c < 3; ++c) out[4 * i + c] = (float) (mean[c] * total);
            out[4 * i + 3] = (float) total;
        }
    }

    // the communicator's id travels through a file next to the scene (any out-of-band channel works:
    // MPI_Bcast, a socket); rank 0 writes it, the other ranks wait for it
    void initComm() {
        uint8_t id[PG_COMM_ID_BYTES];
        fs::path path(m_commIdFile);
        if (m_cfg.rank == 0) {
            check(pg_comm_unique_id(id));
            ref<FileStream> f = new FileStream(path.string() + ".tmp", FileStream::ETruncWrite);
            f->write(id, sizeof(id));
            f->close();
            fs::rename(path.string() + ".tmp", path);
        } else {
            while (!fs::exists(path)) std::this_thread::sleep_for(std::chrono::milliseconds(10));
            ref<FileStream> f = new FileStream(path, FileStream::EReadOnly);
            f->read(id, sizeof(id));
        }
        check(pg_comm_init(m_ctx, id));                          // collective over all ranks
    }

    struct Flattened {
        pg_scene_desc desc;
        std::vector<float> pos, nrm;
        std::vector<uint32_t> idx;
        std::vector<pg_shape> shapes;
        std::vector<pg_material> mats;
        std::vector<pg_emitter> ems;
        std::vector<float> envRGB;            // environment emitter, float RGB, latitude-longitude
        pg_envmap env;
        std::vector<pg_medium> media;
        std::vector<std::vector<float>> densities;  // per medium, [z][y][x], values in [0, 1]
        bool mirrorX = false, hasEnv = false;
        void bind() {  // pg_upload_scene copies everything; the arrays live until then
            desc.num_vertices = (uint32_t) (pos.size() / 3);
            desc.num_triangles = (uint32_t) (idx.size() / 3);
            desc.num_shapes = (uint32_t) shapes.size();
            desc.num_materials = (uint32_t) mats.size();
            desc.num_emitters = (uint32_t) ems.size();
            desc.num_media = (uint32_t) media.size();
            desc.positions = pos.data();
            desc.normals = nrm.data();
            desc.indices = idx.data();
            desc.shapes = shapes.data();
            desc.materials = mats.data();
            desc.emitters = ems.data();
            for (size_t m = 0; m < media.size(); ++m) media[m].density = densities[m].data();
            desc.media = media.empty() ? NULL : media.data();
            env.rgb = envRGB.data();
            desc.envmap = hasEnv ? &env : NULL;
        }
    };
    Flattened flatten(const Scene *scene) const;
    pg_material material(const BSDF *bsdf) const;
    void flattenEnvironment(const Scene *scene, Flattened &f) const;
    int32_t flattenMedium(const Medium *medium, const AABB &bounds, Flattened &f,
                          std::map<const Medium *, int32_t> &index) const;

    pg_config m_cfg;
    void *m_ctx = NULL;
    Flattened m_flat;
    ref<SamplingIntegrator> m_cpu;
    int m_trainingIterations;
    Float m_maxRenderTime;
    std::string m_commIdFile, m_exchange;
    int m_mediumResolution;
    std::string m_sampleCombination, m_denoiserFile;
    bool m_denoise = false;
    struct FilmSums { std::vector<float> rgbw, sumsq; };
    std::vector<FilmSums> m_iterationFilms;                     // sampleCombination = "inversevar"
};

static inline void pgRGB(const Spectrum &s, float *out) {
    Float r, g, b;
    s.toLinearRGB(r, g, b);
    out[0] = (float) r; out[1] = (float) g; out[2] = (float) b; out[3] = 0.0f;
}

// BSDF -> pg_material: the model from BSDF::getModel() (bsdf.h:287-301), the parameters from the
// plugin's own Properties (ConfigurableObject::getProperties, cobject.h:77) with each plugin's defaults
inline pg_material GuidedGPUIntegrator::material(const BSDF *bsdf) const {
    pg_material m;
    memset(&m, 0, sizeof(m));
    if (bsdf->getClass()->getName() == "TwoSidedBRDF") {    // twosided.cpp: the nested BSDF on both sides
        m = material(bsdf->getNestedBSDF(0).get());
        m.flags |= PG_MAT_TWOSIDED;
        return m;
    }
    const Properties &p = bsdf->getProperties();
    auto rough = [&]() {
        std::string d = p.getString("distribution", "beckmann");
        if (d != "beckmann" && d != "ggx") Log(EError, "guided_gpu: distribution '%s' is not supported", d.c_str());
        m.distribution = d == "ggx" ? PG_DIST_GGX : PG_DIST_BECKMANN;
        Float a = p.getFloat("alpha", 0.1f);
        m.alpha_u = (float) p.getFloat("alphaU", a);
        m.alpha_v = (float) p.getFloat("alphaV", a);
        if (!p.getBoolean("sampleVisible", true)) m.flags |= PG_MAT_SAMPLE_ALL;
    };
    switch (bsdf->getModel()) {
        case BSDF::EMSmoothDiffuse:                           // diffuse.cpp:69-80
            m.type = PG_BSDF_DIFFUSE;
            pgRGB(p.getSpectrum("reflectance", Spectrum(0.5f)), m.diffuse_reflectance);
            break;
        case BSDF::EMConductor:
        case BSDF::EMRoughConductor: {                        // (rough)conductor.cpp: material / eta / k / extEta
            m.type = bsdf->getModel() == BSDF::EMConductor ? PG_BSDF_CONDUCTOR : PG_BSDF_ROUGHCONDUCTOR;
            if (m.type == PG_BSDF_ROUGHCONDUCTOR) rough();
            std::string name = boost::to_lower_copy(p.getString("material", "Cu"));
            Spectrum eta, k;
            if (name == "none") {
                eta = Spectrum(0.0f);
                k = Spectrum(1.0f);
            } else {                                          // roughconductor.cpp:173-188, same spectral data
                ref<FileResolver> fr = Thread::getThread()->getFileResolver();
                eta.fromContinuousSpectrum(InterpolatedSpectrum(fr->resolve("data/ior/" + name + ".eta.spd")));
                k.fromContinuousSpectrum(InterpolatedSpectrum(fr->resolve("data/ior/" + name + ".k.spd")));
            }
            Float ext = lookupIOR(p, "extEta", "air");
            pgRGB(p.getSpectrum("eta", eta) / ext, m.eta);
            pgRGB(p.getSpectrum("k", k) / ext, m.k);
            pgRGB(p.getSpectrum("specularReflectance", Spectrum(1.0f)), m.specular_reflectance);
            break;
        }
        case BSDF::EMDielectric:
        case BSDF::EMRoughDielectric:                         // (rough)dielectric.cpp: intIOR bk7, extIOR air
            m.type = bsdf->getModel() == BSDF::EMDielectric ? PG_BSDF_DIELECTRIC : PG_BSDF_ROUGHDIELECTRIC;
            if (m.type == PG_BSDF_ROUGHDIELECTRIC) rough();
            m.int_ior = (float) lookupIOR(p, "intIOR", "bk7");
            m.ext_ior = (float) lookupIOR(p, "extIOR", "air");
            pgRGB(p.getSpectrum("specularReflectance", Spectrum(1.0f)), m.specular_reflectance);
            pgRGB(p.getSpectrum("specularTransmittance", Spectrum(1.0f)), m.specular_transmittance);
            break;
        case BSDF::EMPlastic:
        case BSDF::EMRoughPlastic:                            // (rough)plastic.cpp: polypropylene / air
            m.type = bsdf->getModel() == BSDF::EMPlastic ? PG_BSDF_PLASTIC : PG_BSDF_ROUGHPLASTIC;
            if (m.type == PG_BSDF_ROUGHPLASTIC) rough();
            m.int_ior = (float) lookupIOR(p, "intIOR", "polypropylene");
            m.ext_ior = (float) lookupIOR(p, "extIOR", "air");
            pgRGB(p.getSpectrum("diffuseReflectance", Spectrum(0.5f)), m.diffuse_reflectance);
            pgRGB(p.getSpectrum("specularReflectance", Spectrum(1.0f)), m.specular_reflectance);
            if (p.getBoolean("nonlinear", false)) m.flags |= PG_MAT_NONLINEAR;
            break;
        default:
            if (bsdf->getClass()->getName() == "NullBSDF") { m.type = PG_BSDF_NULL; break; }
            Log(EError, "guided_gpu: BSDF %s is not on the GPU path's BSDF set", bsdf->getClass()->getName().c_str());
    }
    return m;
}

// The environment emitter (Scene::getEnvironmentEmitter, scene.h): envmap.cpp's level-0 bitmap as
// float RGB (latitude-longitude, row 0 at theta = 0), the rotation of toWorld and `scale`
// (envmap.cpp:100-190); a constant emitter (constant.cpp:49) becomes a uniform bitmap.  The library
// builds the sampling CDFs itself (EnvironmentMap::configure, envmap.cpp:260-329).
inline void GuidedGPUIntegrator::flattenEnvironment(const Scene *scene, Flattened &f) const {
    const Emitter *env = scene->getEnvironmentEmitter();
    if (!env) return;
    const Properties &p = env->getProperties();
    const std::string cls = env->getClass()->getName();
    ref<Bitmap> bmp;
    float scale = 1.0f;
    if (cls == "EnvironmentMap") {
        if (p.hasProperty("bitmap"))
            bmp = reinterpret_cast<Bitmap *>(p.getData("bitmap").ptr);       // raw data from another plugin
        else
            bmp = new Bitmap(Thread::getThread()->getFileResolver()->resolve(p.getString("filename")));
        if (p.getFloat("gamma", 0) != 0)
            Log(EError, "guided_gpu: envmap gamma override is not supported (give linear data)");
        scale = (float) p.getFloat("scale", 1.0f);
    } else if (cls == "ConstantBackgroundEmitter") {                          // constant.cpp
        bmp = new Bitmap(Bitmap::ERGB, Bitmap::EFloat32, Vector2i(32, 16));
        Float r, g, b;
        p.getSpectrum("radiance", Spectrum::getD65()).toLinearRGB(r, g, b);
        float *d = bmp->getFloat32Data();
        for (int i = 0; i < 32 * 16; ++i) { d[3 * i] = (float) r; d[3 * i + 1] = (float) g; d[3 * i + 2] = (float) b; }
    } else {
        Log(EError, "guided_gpu: environment emitter %s is not supported (bake it into an envmap)", cls.c_str());
    }
    bmp = bmp->convert(Bitmap::ERGB, Bitmap::EFloat32);
    const Vector2i size = bmp->getSize();
    f.envRGB.assign(bmp->getFloat32Data(), bmp->getFloat32Data() + 3 * (size_t) size.x * size.y);
    memset(&f.env, 0, sizeof(f.env));
    f.env.width = (uint32_t) size.x;
    f.env.height = (uint32_t) size.y;
    const Matrix4x4 M = env->getWorldTransform()->eval(0).getMatrix();
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) f.env.to_world[3 * r + c] = (float) M(r, c);
    f.env.scale = scale;
    f.hasEnv = true;
}

// A participating medium -> pg_medium (index into f.media, memoised).  pg_medium is a density grid
// in [0, 1] times `scale` over an AABB with a constant albedo and an HG phase function:
//   homogeneous (isHomogeneous): a constant 2^3 grid over the scene bounds, scale = sigma_t (grey);
//   heterogeneous (HeterogeneousMedium): the fork's per-point queries (medium.h:168-190,
//     getSigmaT(p) / getScale() = the density, getAlbedo(p)) sampled at the nodes of a
//     mediumResolution^3 grid over the AABB of the medium's boundary shapes -- exact for a
//     GridDataSource of that resolution and AABB (GridDataSource::lookupFloat interpolates nodes,
//     gridvolume.cpp:337-380), a trilinear resampling otherwise;
//   the phase function: HGPhaseFunction's g (hg.cpp:47-50), isotropic = 0.
inline int32_t GuidedGPUIntegrator::flattenMedium(const Medium *med, const AABB &bounds, Flattened &f,
                                                  std::map<const Medium *, int32_t> &index) const {
    if (!med) return -1;
    auto it = index.find(med);
    if (it != index.end()) return it->second;
    pg_medium pm;
    memset(&pm, 0, sizeof(pm));
    pm.type = PG_MEDIUM_HETEROGENEOUS;
    std::vector<float> dens;
    const PhaseFunction *phase = med->getPhaseFunction();
    const std::string pcls = phase ? phase->getClass()->getName() : "IsotropicPhaseFunction";
    if (pcls == "HGPhaseFunction") pm.g = (float) phase->getProperties().getFloat("g", 0.8f);
    else if (pcls == "IsotropicPhaseFunction") pm.g = 0.0f;
    else Log(EError, "guided_gpu: phase function %s is not supported (hg, isotropic)", pcls.c_str());
    if (med->isHomogeneous()) {
        const Spectrum st = med->getSigmaT(), alb = med->getAlbedo();
        if (st.max() != st.min()) Log(EError, "guided_gpu: chromatic sigmaT is not supported");
        for (int a = 0; a < 3; ++a) {
            pm.aabb_min[a] = (float) (bounds.min[a] - bounds.getExtents()[a]);
            pm.aabb_max[a] = (float) (bounds.max[a] + bounds.getExtents()[a]);
        }
        pm.res[0] = pm.res[1] = pm.res[2] = 2;
        dens.assign(8, 1.0f);
        pm.scale = (float) st[0];
        pgRGB(alb, pm.albedo);
    } else {
        const int R = m_mediumResolution;
        const Float scale = med->getScale();
        for (int a = 0; a < 3; ++a) {
            pm.aabb_min[a] = (float) bounds.min[a];
            pm.aabb_max[a] = (float) bounds.max[a];
            pm.res[a] = (uint32_t) R;
        }
        dens.resize((size_t) R * R * R);
        const Vector ext = bounds.getExtents();
        for (int z = 0; z < R; ++z)
            for (int y = 0; y < R; ++y)
                for (int x = 0; x < R; ++x) {
                    const Point q = bounds.min + Vector(ext.x * x / (R - 1), ext.y * y / (R - 1), ext.z * z / (R - 1));
                    dens[((size_t) z * R + y) * R + x] = (float) (med->getSigmaT(q).average() / scale);
                }
        const Spectrum alb = med->getAlbedo(bounds.getCenter());
        for (int k = 0; k < 8; ++k)                       // the GPU medium has one albedo: check the corners
            if (!(med->getAlbedo(bounds.getCorner(k)) == alb) && med->getSigmaT(bounds.getCorner(k)).max() > 0)
                Log(EError, "guided_gpu: spatially varying albedo is not supported");
        pm.scale = (float) scale;
        pgRGB(alb, pm.albedo);
    }
    f.densities.push_back(dens);
    f.media.push_back(pm);
    return index[med] = (int32_t) f.media.size() - 1;
}

inline GuidedGPUIntegrator::Flattened GuidedGPUIntegrator::flatten(const Scene *scene) const {
    Flattened f;
    memset(&f.desc, 0, sizeof(f.desc));
    std::map<const BSDF *, uint32_t> matIndex;
    std::map<const Medium *, AABB> mediumBounds;             // AABB of each medium's boundary shapes
    for (const Shape *shape : scene->getShapes())
        for (const Medium *m : {shape->getInteriorMedium(), shape->getExteriorMedium()})
            if (m) mediumBounds[m].expandBy(shape->getAABB());
    const AABB sceneBounds = scene->getAABB();
    std::map<const Medium *, int32_t> medIndex;
    auto mediumOf = [&](const Medium *m) {
        return flattenMedium(m, m && !m->isHomogeneous() ? mediumBounds[m] : sceneBounds, f, medIndex);
    };
    if (m_cfg.integrator != PG_INTEGRATOR_VOLPATH && !mediumBounds.empty())
        Log(EError, "guided_gpu: the scene has participating media: use guided_gpu_volpath");
    for (const Shape *shape : scene->getShapes()) {         // ref_vector<Shape>, scene.h:1084-1086
        // TriMesh as is; spheres, rectangles, disks, cubes ... through Shape::createTriMesh (shape.h:230)
        ref<TriMesh> mesh = shape->getClass()->derivesFrom(MTS_CLASS(TriMesh))
            ? static_cast<TriMesh *>(const_cast<Shape *>(shape)) : const_cast<Shape *>(shape)->createTriMesh();
        if (!mesh) Log(EError, "guided_gpu: shape %s has no triangle mesh", shape->getClass()->getName().c_str());
        const BSDF *bsdf = shape->getBSDF();
        if (!matIndex.count(bsdf)) {
            matIndex[bsdf] = (uint32_t) f.mats.size();
            f.mats.push_back(material(bsdf));
        }
        pg_shape s;
        s.tri_begin = (uint32_t) (f.idx.size() / 3);
        s.tri_count = (uint32_t) mesh->getTriangleCount();
        s.material = matIndex[bsdf];
        s.emitter = -1;
        s.interior_medium = mediumOf(shape->getInteriorMedium());   // Shape::getTargetMedium semantics
        s.exterior_medium = mediumOf(shape->getExteriorMedium());
        if (shape->isEmitter()) {                            // AreaLight (area.cpp:62-90): radiance
            pg_emitter e;
            memset(&e, 0, sizeof(e));
            e.shape = (uint32_t) f.shapes.size();
            pgRGB(shape->getEmitter()->getProperties().getSpectrum("radiance"), e.radiance);
            s.emitter = (int32_t) f.ems.size();
            f.ems.push_back(e);
        }
        const Point *P = mesh->getVertexPositions();         // trimesh.h:122-141, world space
        const Normal *N = mesh->getVertexNormals();
        const Triangle *T = mesh->getTriangles();
        if (N) {                                             // shared vertices with shading normals
            const uint32_t base = (uint32_t) (f.pos.size() / 3);
            for (size_t v = 0; v < mesh->getVertexCount(); ++v)
                for (int a = 0; a < 3; ++a) {
                    f.pos.push_back((float) P[v][a]);
                    f.nrm.push_back((float) N[v][a]);
                }
            for (size_t t = 0; t < mesh->getTriangleCount(); ++t)
                for (int k = 0; k < 3; ++k) f.idx.push_back(base + T[t].idx[k]);
        } else {                                             // no normals: Mitsuba shades with the face normal
            for (size_t t = 0; t < mesh->getTriangleCount(); ++t) {
                const Point &a = P[T[t].idx[0]], &b = P[T[t].idx[1]], &c = P[T[t].idx[2]];
                const Normal n(normalize(cross(b - a, c - a)));
                for (int k = 0; k < 3; ++k) {
                    const Point &q = P[T[t].idx[k]];
                    for (int ax = 0; ax < 3; ++ax) {
                        f.pos.push_back((float) q[ax]);
                        f.nrm.push_back((float) n[ax]);
                    }
                    f.idx.push_back((uint32_t) (f.pos.size() / 3 - 1));
                }
            }
        }
        f.shapes.push_back(s);
    }
    // PerspectiveCamera (perspective.cpp): toWorld at t = 0, fov along x, clip planes; its medium
    const PerspectiveCamera *cam = dynamic_cast<const PerspectiveCamera *>(scene->getSensor());
    if (!cam) Log(EError, "guided_gpu: only the perspective sensor is supported");
    const Transform T = cam->getWorldTransform()->eval(0);
    const Point o = T(Point(0.0f)), tgt = T(Point(0, 0, 1));
    const Vector up = T(Vector(0, 1, 0));
    f.mirrorX = T.getMatrix().det3x3() < 0;                 // mirrored toWorld (Blender exports): flip read-out
    pg_camera &c = f.desc.camera;
    for (int a = 0; a < 3; ++a) {
        c.origin[a] = (float) o[a];
        c.target[a] = (float) tgt[a];
        c.up[a] = (float) up[a];
    }
    c.fov_x_deg = (float) cam->getXFov();
    c.near_clip = (float) cam->getNearClip();
    c.far_clip = (float) cam->getFarClip();
    c.width = (uint32_t) cam->getFilm()->getSize().x;
    c.height = (uint32_t) cam->getFilm()->getSize().y;
    f.desc.camera_medium = mediumOf(cam->getMedium());
    flattenEnvironment(scene, f);
    return f;  // the caller binds the descriptor's pointers (Flattened::bind) to its own copy
}

MTS_NAMESPACE_END
