// Timing events for the live kernel probe (bench.py roofline, tools/layer_report.py).
//
// A default hipEvent record ends with a system-scope release: the L2 is written back and invalidated, so the kernel
// launched after it starts from cold caches and an event pair around every conv launch measures each conv colder
// than it runs in the captured step.  These events are created with hipEventDisableSystemFence: the record is only
// a timestamp on the stream, the caches stay as the previous kernel left them.  Elapsed times are read after a
// stream/device synchronisation (the probe never inspects the events before that), which is what the flag asks.
#include "common.h"

extern "C" int ssseg_probe_event_create(void** ev_out)
{
    if (!ev_out) return SSSEG_EINVAL;
    hipEvent_t e = nullptr;
    hipError_t rc = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
    if (rc != hipSuccess) return (int)rc;
    *ev_out = (void*)e;
    return SSSEG_OK;
}

extern "C" int ssseg_probe_event_record(void* ev, ssseg_stream_t stream)
{
    if (!ev) return SSSEG_EINVAL;
    return (int)hipEventRecord((hipEvent_t)ev, (hipStream_t)stream);
}

extern "C" int ssseg_probe_event_elapsed(void* ev0, void* ev1, float* ms_out)
{
    if (!ev0 || !ev1 || !ms_out) return SSSEG_EINVAL;
    hipError_t rc = hipEventSynchronize((hipEvent_t)ev1);
    if (rc != hipSuccess) return (int)rc;
    return (int)hipEventElapsedTime(ms_out, (hipEvent_t)ev0, (hipEvent_t)ev1);
}

extern "C" int ssseg_probe_event_destroy(void* ev)
{
    if (!ev) return SSSEG_OK;
    return (int)hipEventDestroy((hipEvent_t)ev);
}
