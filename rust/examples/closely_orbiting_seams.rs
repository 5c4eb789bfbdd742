//! testscene_closelyOrbitingSphere's loop (main.rs:1468-1633) one seam at a time, as
//! the reference writes it: per frame a shadow viewport (ORTHOGONAL, face BACK)
//! rasterized and ray-marched, an eye viewport (face FRONT) rasterized, then
//! renderColorImage and writeColorImage.  Each seam is one librtm call on the
//! device (the zBuffers and G-buffers stay there); Context::render is the same frame
//! in one call, and examples/closely_orbiting.rs the batched animation.
use rtm::rtm_ffi::*;
use rtm::{render_color_image, Camera, Context, Error, Scene};

fn scene(frame: i32) -> Scene {
    let f = frame as f64;
    Scene {
        // main.rs:1475-1522
        spheres: vec![
            rtm_sphere { id: 0, pos: [0.0, 0.0, 0.5], r: 0.2, color: [0.02, 0.02, 1.0] },
            rtm_sphere { id: 1, pos: [0.0, 0.0, 0.5 + 0.2 * 2.0], r: 0.2, color: [0.02, 0.02, 1.0] },
            rtm_sphere { id: 2, pos: [-0.0, (f * 0.025).sin() * 0.7, (f * 0.025).cos() * 0.7], r: 0.1,
                         color: [0.9, 0.2, 0.2] },
        ],
        // rayEntry_ShadowRay_testing's patch (main.rs:2024-2029)
        patches: vec![rtm_patch { a0: 0.1, b0: 0.1, a1: 0.1, b1: 0.1 }],
        ..Scene::default()
    }
}

fn main() -> Result<(), Error> {
    let (w, h, steps) = (512, 512, 500); // the reference's viewports and march (main.rs:1534, 2031)
    let sun: Camera = rtm_camera { type_: RTM_CAMERA_ORTHOGONAL, reserved: 0, pos: [0.0, 0.0, 0.0],
                                   dir: [0.0, 0.0, 1.0], up: [0.0, 1.0, 0.0], side: [1.0, 0.0, 0.0] };
    let eye: Camera = rtm_camera { type_: RTM_CAMERA_ORTHOGONAL, reserved: 0, pos: [-1.0, 0.0, 0.0],
                                   dir: [1.0, 0.0, 0.0], up: [0.0, 1.0, 0.0], side: [0.0, 0.0, 1.0] };
    let ctx = Context::new(0)?;
    for frame_number in 0..300 {
        let scene = scene(frame_number);
        // viewport for shadow mapping (main.rs:1532-1566)
        let mut viewport1 = ctx.viewport(w, h, RTM_FACE_BACK, &sun)?;
        viewport1.rasterize(&scene)?;
        viewport1.process_raymarching_rays(&scene.patches, steps)?;
        // normal rendering (main.rs:1580-1616)
        let mut viewport0 = ctx.viewport(w, h, RTM_FACE_FRONT, &eye)?;
        viewport0.rasterize(&scene)?;
        // (*) render color image, (*) write image (main.rs:1626-1630)
        let image = render_color_image(&scene, &viewport0, &viewport1)?;
        // the one-call frame is the same image, bit for bit
        debug_assert!(ctx.render(&scene, &eye, &sun, w, h, steps, 0)?.iter().zip(&image)
                          .all(|(a, b)| a.to_bits() == b.to_bits()));
        let text = ppm_p3(&image, w, h);
        std::fs::write(format!("img{:06}.ppm", frame_number), text).expect("write ppm");
    }
    Ok(())
}

/// writeColorImage (main.rs:660-704) on the host for a host image: "P3\n{W} {H}\n255\n"
/// then "{r} {g} {b}  " per pixel and "\n" per row, each channel
/// (max(0).min(1) ^ (1/2.2) * 255) as i64.  (Context::ppm_text generates the same text on
/// the GPU from a device frame.)
fn ppm_p3(img: &[f32], w: i32, h: i32) -> String {
    let mut s = format!("P3\n{} {}\n255\n", w, h);
    for y in 0..h as usize {
        for x in 0..w as usize {
            let p = &img[(y * w as usize + x) * 4..][..3];
            let b = |c: f32| (f32::powf(c.max(0.0).min(1.0), 1.0f32 / 2.2f32) * 255.0) as i64;
            s.push_str(&format!("{} {} {}  ", b(p[0]), b(p[1]), b(p[2])));
        }
        s.push('\n');
    }
    s
}
