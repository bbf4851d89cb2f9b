"""The reference's own instance, end to end, through its own call shape.

src/main.cpp renders WIDTH x HEIGHT = 440 x 330 (main.cpp:29-30) with NUM_SHAPES 10 and AA 4
(main.cpp:31-36), myscene = scene1 (main.cpp:146: 4 spheres + a plane, src/scene.h:15-65) and
lighting = 1 (main.cpp:309): every frame compute() (main.cpp:553-560) refills rand_buffer and
calls compute_two_shaders(frame, aop_compute, aop_postprocessing) (main.cpp:622-671), which
copies the whole 55,757,840-byte shader_data SSBO to the GPU, dispatches both programs over
440 x 330 and copies the whole SSBO back.  Here the same 12 frames go through
rt_compute_two_shaders with the whole host SSBO in and out, and the oracle re-executes them
on its own copy: the whole image and the whole SSBO (header, shapes, rand_buffer and the
8-slot pixels / normals / depth ring) are compared.  440 and 330 are not multiples of the
kernels' 16-px pools and tiles, so the partial pools and tiles at the edges run too.
"""
import numpy as np
import pytest

import oracle
from conftest import assert_bitwise, assert_close
from real_time_ray_tracer_amd import AOP_COMPUTE, AOP_POSTPROCESSING, SSBO, Header, Renderer
from real_time_ray_tracer_amd.host import ssbo_floats

pytestmark = pytest.mark.gpu

W, H, NUM_SHAPES, AA = 440, 330, 10, 4  # src/main.cpp:29-36
ASPECT = 1.333333                       # ASPECT_RATIO, src/main.cpp:39


def test_reference_instance_twelve_frames_through_compute_two_shaders():
    h = Header.builtin(1, AA, ASPECT, num_shapes=NUM_SHAPES)
    assert h.num_objects == 5  # true_num_scene_objects of scene1
    sg, so = SSBO(h, W, H), SSBO(h, W, H)
    assert sg.data.nbytes == 4 * ssbo_floats(NUM_SHAPES, AA, W, H) == 55_757_840
    r = Renderer(W, H, NUM_SHAPES, AA)
    d = oracle.dims(W, H, NUM_SHAPES, AA)
    ig, io = np.zeros((H, W, 4), np.float32), np.zeros((H, W, 4), np.float32)
    fg = fo = 0
    for k in range(12):
        h.fill_rand_buffer(7000 + k)  # fill_rand_buffer() (seeded), main.cpp:535-539
        sg.set_header(h)
        so.set_header(h)
        so.data[1] = sg.data[1]  # mode.y is the dispatch's own write (main.cpp:626); keep both equal
        fg = r.compute_two_shaders(sg, fg, AOP_COMPUTE, AOP_POSTPROCESSING, ig)
        oracle.run_program(so.data, d, oracle.AOP_COMPUTE, fo, io)
        oracle.run_program(so.data, d, oracle.AOP_POSTPROCESSING, fo, io)
        fo = (fo + 1) % 8
        assert fg == fo
        h.data[:] = sg.data[:h.data.size]  # the SSBO copied back is the next frame's host state
    r.close()
    assert_close(ig, io, "image")
    hn = h.data.size
    assert_bitwise(sg.data[:hn], so.data[:hn], "header + shapes + rand_buffer")
    assert_close(sg.pixels, so.pixels, "pixels ring")
    assert_bitwise(sg.normals, so.normals, "normals ring")
    assert_bitwise(sg.depth, so.depth, "depth ring")
    assert_close(sg.data, so.data, "whole SSBO")
    # every slot of the ring holds a rendered frame (12 frames > 8 slots): nothing left at zero
    assert (np.abs(sg.pixels).sum(axis=(1, 2, 3)) > 0).all()
