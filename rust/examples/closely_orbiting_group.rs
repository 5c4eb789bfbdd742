//! testscene_closelyOrbitingSphere (main.rs:1468-1633) on every GPU of the node: each
//! frame tile-partitioned over the devices and gathered by RCCL (Group, INTEGRATION.md
//! §3c), returned as writeColorImage's RGB8 bytes (main.rs:660-704) and written as the
//! reference's PPM frames.  The per-frame scene construction is the reference's
//! (main.rs:1475-1522); the frame is the north star's 3840x2160, K = 64.
use rtm::rtm_ffi::*;
use rtm::{Error, Group, Scene};
use std::io::Write;

fn main() -> Result<(), Error> {
    let (w, h, steps) = (3840, 2160, 64);
    let shadow = rtm_camera { type_: RTM_CAMERA_ORTHOGONAL, reserved: 0, pos: [0.0, 0.0, 0.0], dir: [0.0, 0.0, 1.0],
                              up: [0.0, 1.0, 0.0], side: [1.0, 0.0, 0.0] };
    let eye = rtm_camera { type_: RTM_CAMERA_ORTHOGONAL, reserved: 0, pos: [-1.0, 0.0, 0.0], dir: [1.0, 0.0, 0.0],
                           up: [0.0, 1.0, 0.0], side: [0.0, 0.0, 1.0] };
    let group = Group::new(&[])?; // every device of the node, one RCCL communicator
    let mut rgb = Vec::new();
    for frame in 0..300 {
        let f = frame as f64;
        let scene = Scene {
            spheres: vec![
                rtm_sphere { id: 0, pos: [0.0, 0.0, 0.5], r: 0.2, color: [0.02, 0.02, 1.0] },
                rtm_sphere { id: 1, pos: [0.0, 0.0, 0.5 + 0.2 * 2.0], r: 0.2, color: [0.02, 0.02, 1.0] },
                rtm_sphere { id: 2, pos: [-0.0, (f * 0.025).sin() * 0.7, (f * 0.025).cos() * 0.7], r: 0.1,
                             color: [0.9, 0.2, 0.2] },
            ],
            patches: vec![rtm_patch { a0: 0.3, b0: 2.1, a1: 0.9, b1: 2.7 }], // Scene A-bench
            ..Default::default()
        };
        group.render_into(&scene, &eye, &shadow, w, h, steps, 0, RTM_FORMAT_RGB8, &mut rgb)?;
        // writeColorImage's file (main.rs:686-703): P3 text of the same bytes
        let mut out = std::io::BufWriter::new(std::fs::File::create(format!("img{:06}.ppm", frame)).expect("ppm"));
        write!(out, "P3\n{} {}\n255\n", w, h).expect("ppm");
        for row in rgb.chunks(w as usize * 3) {
            for px in row.chunks(3) {
                write!(out, "{} {} {}  ", px[0], px[1], px[2]).expect("ppm");
            }
            writeln!(out).expect("ppm");
        }
    }
    Ok(())
}
