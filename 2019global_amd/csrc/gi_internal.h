// gi_internal.h — declarations shared by the host translation units of libgi (gi_capi.cpp,
// gi_multi.cpp).  Not part of the C-ABI.
#pragma once

#include <hip/hip_runtime_api.h>

#include <exception>
#include <mutex>
#include <new>
#include <string>

#include "gi.h"
#include "gi_scene.h"

namespace gi {

// camera basis and frame corner of raytracer.h:26-30 (the kernels' CamDev, gi_kernels.hip)
struct CamDev {
    V3 pos, up, left, top_left;
    double rx, ry;
};

int error(int code, const std::string& msg) noexcept;      // sets gi_last_error, returns code
int hip_error(hipError_t e, const char* what) noexcept;    // GI_ERR_DEVICE with HIP's message
int bind_device(int device);
int check_device(int device);                              // gfx950 or GI_ERR_DEVICE
CamDev make_cam(const gi_camera& c, int w);
int check_opts(int w, int h, const gi_opts* o);
int band_rows_of(const gi_opts* o, int h);                 // progressive band height (whole tile rows)

int scene_create_on(const gi_scene_desc* desc, int device, gi_scene** out);
void scene_destroy(gi_scene* s) noexcept;
int scene_device(const gi_scene* s);
std::mutex& scene_mutex(gi_scene* s);
int scene_render_band(gi_scene* s, const CamDev& cd, const double light[3], int w, int h, int y0, const gi_opts& o,
                      double* d_rgb, uint8_t* d_rgb8, hipStream_t stream, bool timer);
int unshard(int w, int h, int n, const double* packed, const uint8_t* packed8, double* rgb, uint8_t* rgb8,
            hipStream_t stream);

// Restores the calling thread's current HIP device on scope exit (entry points that switch devices
// leave the caller's choice as they found it).
struct DeviceRestore {
    int dev = -1;
    DeviceRestore() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceRestore() {
        int cur = -1;
        if (dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != dev) (void)hipSetDevice(dev);
    }
    DeviceRestore(const DeviceRestore&) = delete;
    DeviceRestore& operator=(const DeviceRestore&) = delete;
};

// Runs an entry point's body: no exception leaves the library (gi.h).
template <typename F>
int guard(F&& body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return error(GI_ERR_NOMEM, "host memory exhausted");
    } catch (const std::exception& e) {
        return error(GI_ERR_INTERNAL, std::string("internal error: ") + e.what());
    } catch (...) {
        return error(GI_ERR_INTERNAL, "internal error");
    }
}

}  // namespace gi
