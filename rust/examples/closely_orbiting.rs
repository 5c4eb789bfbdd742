//! testscene_closelyOrbitingSphere (main.rs:1468-1633) on the GPU: the reference's
//! 300-frame animation, rendered 64 frames per rtm_render_frames_async call into a
//! swap chain of device frames, every frame written as writeColorImage's PPM.
//! The per-frame scene construction is the reference's (main.rs:1475-1522).
use rtm::rtm_ffi::*;
use rtm::{Context, Error};

fn scene_spheres(frame: i32) -> Vec<rtm_sphere> {
    let f = frame as f64;
    vec![
        rtm_sphere { id: 0, pos: [0.0, 0.0, 0.5], r: 0.2, color: [0.02, 0.02, 1.0] },
        rtm_sphere { id: 1, pos: [0.0, 0.0, 0.5 + 0.2 * 2.0], r: 0.2, color: [0.02, 0.02, 1.0] },
        rtm_sphere { id: 2, pos: [-0.0, (f * 0.025).sin() * 0.7, (f * 0.025).cos() * 0.7], r: 0.1,
                     color: [0.9, 0.2, 0.2] },
    ]
}

fn main() -> Result<(), Error> {
    let (w, h, steps) = (512, 512, 500); // the reference's 512x512 viewports, 500 march steps (main.rs:2031)
    // shadow camera: the sun along +z (main.rs:1552-1563); eye at (-1,0,0) looking along +x (main.rs:1598-1609)
    let shadow = rtm_camera { type_: RTM_CAMERA_ORTHOGONAL, reserved: 0, pos: [0.0, 0.0, 0.0], dir: [0.0, 0.0, 1.0],
                              up: [0.0, 1.0, 0.0], side: [1.0, 0.0, 0.0] };
    let eye = rtm_camera { type_: RTM_CAMERA_ORTHOGONAL, reserved: 0, pos: [-1.0, 0.0, 0.0], dir: [1.0, 0.0, 0.0],
                           up: [0.0, 1.0, 0.0], side: [0.0, 0.0, 1.0] };
    let patch = rtm_patch { a0: 0.1, b0: 0.1, a1: 0.1, b1: 0.1 }; // rayEntry_ShadowRay_testing (main.rs:2024-2029)
    let ctx = Context::new(0)?;
    let segment = 64usize;
    let ring = ctx.alloc_frames(segment, w, h)?;
    let spheres: Vec<Vec<rtm_sphere>> = (0..300).map(scene_spheres).collect();
    for first in (0..300usize).step_by(segment) {
        let n = segment.min(300 - first);
        let scenes: Vec<rtm_scene> = (first..first + n)
            .map(|i| rtm_scene { spheres: spheres[i].as_ptr(), patches: &patch, n_spheres: 3, n_patches: 1,
                                 circle_planes: std::ptr::null(), capped_cylinders: std::ptr::null(),
                                 n_circle_planes: 0, n_capped_cylinders: 0, sdfs: std::ptr::null(), n_sdfs: 0,
                                 reserved: 0 })
            .collect();
        ctx.render_frames(&scenes, &eye, &shadow, w, h, steps, 0, &ring.frames[..n])?;
        for k in 0..n {
            // writeColorImage(&image, "img{:06}.ppm") (main.rs:1630), from the device frame
            let text = ctx.ppm_text(ring.frames[k], w, h)?;
            std::fs::write(format!("img{:06}.ppm", first + k), text).expect("write ppm");
        }
    }
    Ok(())
}
