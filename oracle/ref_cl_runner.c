/*
 * ref_cl_runner.c -- runs the REFERENCE's own GPU kernel (TEST INFRASTRUCTURE
 * ONLY; nothing in the product links it).
 *
 * oracle/Makefile (target `ref`) compiles /root/reference/smith_waterman/src/
 * smith_waterman.cl, where it lies, for gfx950 into the code object
 * oracle/_ref/smith_waterman_gfx950.co (OpenCL C 1.2, the language the
 * reference's `ocl` crate builds at run time, aligner.rs:504-508).  This
 * runner is the reference host path of gpu_align (aligner.rs:410-532)
 * restated over the OpenCL C API instead of the Rust `ocl` crate: the first
 * GPU of the first platform (gpu.rs:112-132), buffers for seq1/seq2/result
 * (aligner.rs:478-499), the program from the prebuilt binary instead of the
 * source (the source does not travel to the GPU box), kernel
 * `smith_waterman_align` with args (seq1, seq2, result, length) and the
 * NDRange global = G * W, local = W (:510-521), blocking finish and a read of
 * the one result int (:527-530).  The reference leaves `result`
 * uninitialised (:494-499); it is zeroed here.
 *
 * Built into oracle/_ref/libref_cl.so; tests/test_gpu_reference_kernel.py
 * compares msw_align_compat (K0) against it on the GPU box.
 */
#define CL_TARGET_OPENCL_VERSION 120
#include <CL/cl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void set_err(char* err, size_t n, const char* what, cl_int code) {
    if (err && n) snprintf(err, n, "%s failed (OpenCL error %d)", what, (int)code);
}

#define CL_CHECK(expr, what)                      \
    do {                                          \
        cl_int e_ = (expr);                       \
        if (e_ != CL_SUCCESS) {                   \
            set_err(err, errlen, what, e_);       \
            rc = -1;                              \
            goto done;                            \
        }                                         \
    } while (0)

/* Runs smith_waterman_align (or, with detailed != 0, smith_waterman_detailed
 * with args (seq1, seq2, result, len1, len2)) once.  Returns 0 on success. */
int ref_cl_run(const char* co_path, int detailed, const uint8_t* s1, uint32_t n1, const uint8_t* s2, uint32_t n2,
               uint32_t wg, uint64_t groups, int32_t* result, char* err, size_t errlen) {
    int rc = 0;
    cl_int e = CL_SUCCESS;
    cl_platform_id plat = NULL;
    cl_device_id dev = NULL;
    cl_context ctx = NULL;
    cl_command_queue q = NULL;
    cl_program prog = NULL;
    cl_kernel k = NULL;
    cl_mem b1 = NULL, b2 = NULL, br = NULL;
    unsigned char* bin = NULL;
    size_t bin_len = 0;
    cl_int bin_status = CL_SUCCESS;
    const int32_t zero = 0;

    FILE* f = fopen(co_path, "rb");
    if (!f) {
        if (err && errlen) snprintf(err, errlen, "cannot open %s", co_path);
        return -1;
    }
    fseek(f, 0, SEEK_END);
    bin_len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    bin = (unsigned char*)malloc(bin_len);
    if (!bin || fread(bin, 1, bin_len, f) != bin_len) {
        fclose(f);
        free(bin);
        if (err && errlen) snprintf(err, errlen, "cannot read %s", co_path);
        return -1;
    }
    fclose(f);

    CL_CHECK(clGetPlatformIDs(1, &plat, NULL), "clGetPlatformIDs");
    CL_CHECK(clGetDeviceIDs(plat, CL_DEVICE_TYPE_GPU, 1, &dev, NULL), "clGetDeviceIDs");
    ctx = clCreateContext(NULL, 1, &dev, NULL, NULL, &e);
    CL_CHECK(e, "clCreateContext");
    q = clCreateCommandQueue(ctx, dev, 0, &e);
    CL_CHECK(e, "clCreateCommandQueue");
    prog = clCreateProgramWithBinary(ctx, 1, &dev, &bin_len, (const unsigned char**)&bin, &bin_status, &e);
    CL_CHECK(e, "clCreateProgramWithBinary");
    CL_CHECK(bin_status, "binary status");
    CL_CHECK(clBuildProgram(prog, 1, &dev, "", NULL, NULL), "clBuildProgram");
    k = clCreateKernel(prog, detailed ? "smith_waterman_detailed" : "smith_waterman_align", &e);
    CL_CHECK(e, "clCreateKernel");
    b1 = clCreateBuffer(ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, n1 ? n1 : 1, (void*)s1, &e);
    CL_CHECK(e, "clCreateBuffer(seq1)");
    b2 = clCreateBuffer(ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, n2 ? n2 : 1, (void*)s2, &e);
    CL_CHECK(e, "clCreateBuffer(seq2)");
    br = clCreateBuffer(ctx, CL_MEM_READ_WRITE | CL_MEM_COPY_HOST_PTR, sizeof(int32_t), (void*)&zero, &e);
    CL_CHECK(e, "clCreateBuffer(result)");
    CL_CHECK(clSetKernelArg(k, 0, sizeof(cl_mem), &b1), "arg seq1");
    CL_CHECK(clSetKernelArg(k, 1, sizeof(cl_mem), &b2), "arg seq2");
    CL_CHECK(clSetKernelArg(k, 2, sizeof(cl_mem), &br), "arg result");
    if (detailed) {
        cl_uint l1 = n1, l2 = n2;
        CL_CHECK(clSetKernelArg(k, 3, sizeof(cl_uint), &l1), "arg len1");
        CL_CHECK(clSetKernelArg(k, 4, sizeof(cl_uint), &l2), "arg len2");
    } else {
        cl_uint len = n1 < n2 ? n1 : n2; /* aligner.rs:413 */
        CL_CHECK(clSetKernelArg(k, 3, sizeof(cl_uint), &len), "arg length");
    }
    {
        size_t local = wg, global = (size_t)groups * wg;
        CL_CHECK(clEnqueueNDRangeKernel(q, k, 1, NULL, &global, &local, 0, NULL, NULL), "clEnqueueNDRangeKernel");
    }
    CL_CHECK(clFinish(q), "clFinish");
    CL_CHECK(clEnqueueReadBuffer(q, br, CL_TRUE, 0, sizeof(int32_t), result, 0, NULL, NULL), "read result");
done:
    if (b1) clReleaseMemObject(b1);
    if (b2) clReleaseMemObject(b2);
    if (br) clReleaseMemObject(br);
    if (k) clReleaseKernel(k);
    if (prog) clReleaseProgram(prog);
    if (q) clReleaseCommandQueue(q);
    if (ctx) clReleaseContext(ctx);
    free(bin);
    return rc;
}
