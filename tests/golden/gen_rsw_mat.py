"""Extract the MATLAB-produced arrays of the reference's `rsw/matlab.mat` into a
small committed fixture (tests/golden/rsw_matlab.npz), and copy the
reference's appended `pv_time.bin` (qg_flow_ray_trace/data/.nfs00000000032a756700000024)
to tests/golden/pv_time_ref.bin.

These are the only numeric outputs of MATLAB itself that the reference holds
(VERDICT r1 "What's missing" #1).  `matlab.mat` is the workspace of
an `rsw/swk.m` run (R2020b FFTW): at the saved instant

  * `Sk`   (255x128x3 complex) is the spectral state [uk vk hk] in g2k's
    half-plane layout (swk.m:113 g2k, :182 AB3 update);
  * `u`, `v`, `h` = k2gp(Sk(:,:,i)) (swk.m:205-207) — their REAL parts are
    nx^2*ifft2(ifftshift(fulspec(damask.*Sk))) on the grid (the imaginary part
    holds the dx/2-shifted field of the dealiasing trick, k2gp swk.m:221-230);
  * `zeta` = k2gp(ikx_.*Sk(:,:,2) - iky_.*Sk(:,:,1)) (swk.m:209);
  * `divuk` = ikx_.*Sk(:,:,1) + iky_.*Sk(:,:,2) (swk.m:210);
  * `ikx_`, `iky_` = 1i*kx_, 1i*ky_ of ndgrid(-kmax:kmax, 0:kmax);
  * `Sin` (256x256x3) the run's initial grid state and `Sout(:,:,:,1:4)` the
    saved frames k2g(Sk) (swk.m:146, k2g = swk.m:282-288, the same
    nx^2*ifft2(ifftshift(fulspec(.))) as qg_flow_ray_trace/k2g.m): frame 1 is
    k2g(g2k(Sin)) (swk.m:113), frame 4 is k2g of the saved `Sk` above.

The saved state is a one-dimensional wave (only the ky = 0 line of Sk is
non-zero; every field depends on x alone), so these arrays pin, on the ky = 0
line, g2k.m / k2g.m / fulspec.m's row layout, fftshift, 1/nx^2 normalisation, the
kx < 0 conjugate completion of fulspec.m:16, the first-index = x axis
convention, and the i*kx derivative convention of grid_U.m:2-9 and
SpectralScheme.m:16-25 against MATLAB's own FFT.  The same state is the
realistic RSW background of ray_trace_sw/raytrace_sw.m:25-52 (S(:,:,1:3) =
[u v eta], f = Cg = 1, L = 2*pi), whose restart file is not in the reference
(.MISSING_LARGE_BLOBS).

Only data is read (scipy.io.loadmat, no code execution).  Run here, where
/root/reference exists:  python tests/golden/gen_rsw_mat.py
"""
import os
import shutil

import numpy as np
import scipy.io

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
MAT = os.path.join(REF, "rsw", "matlab.mat")
PV_TIME = os.path.join(REF, "qg_flow_ray_trace", "data", ".nfs00000000032a756700000024")


def main():
    m = scipy.io.loadmat(MAT)
    nx = int(m["nx"][0, 0])
    kmax = int(m["kmax"][0, 0])
    # the wavenumber operators MATLAB stored are exactly i*ndgrid(-kmax:kmax, 0:kmax)
    kx_, ky_ = np.meshgrid(np.arange(-kmax, kmax + 1), np.arange(0, kmax + 1), indexing="ij")
    assert np.array_equal(m["ikx_"], 1j * kx_) and np.array_equal(m["iky_"], 1j * ky_)
    out = dict(
        nx=np.int64(nx),
        kmax=np.int64(kmax),
        f=np.float64(m["f"][0, 0]),
        Cg=np.float64(m["Cg"][0, 0]),
        L=np.float64(m["L"][0, 0]),
        dx=np.float64(m["dx"][0, 0]),
        Sk=np.asarray(m["Sk"], dtype=np.complex128),
        u=np.ascontiguousarray(m["u"].real),
        v=np.ascontiguousarray(m["v"].real),
        h=np.ascontiguousarray(m["h"].real),
        zeta=np.ascontiguousarray(m["zeta"].real),
        divuk=np.asarray(m["divuk"], dtype=np.complex128),
        ikx_imag=np.asarray(m["ikx_"].imag, dtype=np.int16),
        iky_imag=np.asarray(m["iky_"].imag, dtype=np.int16),
        Sin=np.asarray(m["Sin"], dtype=np.float64),
        Sout=np.ascontiguousarray(m["Sout"][:, :, :, :4]),
        time=np.asarray(m["time"][0, :4], dtype=np.float64),
    )
    np.savez_compressed(os.path.join(HERE, "rsw_matlab.npz"), **out)
    shutil.copyfile(PV_TIME, os.path.join(HERE, "pv_time_ref.bin"))
    print("wrote rsw_matlab.npz and pv_time_ref.bin")


if __name__ == "__main__":
    main()
