"""Faults behind the uploads' pinned staging ring are reported, not swallowed (VERDICT r5 weak
item 6).  The reference's upload is a plain memcpy into the mapped SSBO (src/main.cpp:598-602);
here each rt_upload_header goes through one of 8 pinned buffers whose "consumed" event is
queried before the buffer is reused.  Only hipErrorNotReady means "still in use"; any other
result of that query must come back as RT_E_HIP with the HIP code, and the buffer must not be
reused under a failed copy."""
import pytest

from real_time_ray_tracer_amd import Header, Renderer, RtError, aspect_for

pytestmark = pytest.mark.gpu

HIP_ERROR_LAUNCH_FAILURE = 719


def test_failed_staging_query_is_returned():
    W, H, spp = 64, 48, 4
    h = Header.synthetic(8, spp, 5, aspect_for(W, H))
    r = Renderer(W, H, h.S, h.AA)
    try:
        f = 0
        for k in range(8):  # every slot of the staging ring used once: the next upload queries one
            h.fill_rand_buffer(7000 + k)
            h.set_mode(f, h.num_objects)
            r.upload_header(h)
            f = r.dispatch(2, f)
        r.synchronize()
        r.debug_fail_next_event_query(HIP_ERROR_LAUNCH_FAILURE)
        with pytest.raises(RtError) as e:
            r.upload_header(h)
        assert e.value.status == -3 and e.value.hip == HIP_ERROR_LAUNCH_FAILURE, str(e.value)
        # the hook fires once: the next upload queries HIP again and goes through
        r.upload_header(h)
        r.dispatch(2, f)
        r.synchronize()
        with pytest.raises(RtError):
            r.debug_fail_next_event_query(0)  # hipSuccess is not a fault
    finally:
        r.close()
