function [x, k, t_end] = trace_stored_gpu(pv_path, nx, x, k, f, Cg, opts)
% Packets through a stored PV series on the MI355X (BASELINE configs[2]):
% the stored-field consumer's read_field -> g2k -> grid_U
% (symplectic_full_fourier.m:18-20, read_field.m, g2k.m:8-9, grid_U.m:1-18)
% for every frame, with both transforms on the device (swrt_set_field_q),
% and interpolate_U's linear blend between consecutive frames
% (interpolate_U.m:19-23) advanced by opts.nsub leapfrog substeps per
% interval, up to four intervals per call (swrt_advance_intervals: the same
% bits as one call per interval).  x, k: N x 2.  opts (all optional):
% frames (default: every frame of pv_path.bin), times (default: pv_time.bin
% beside it), nlayers (1; 2 traces layer 1 with the 2-layer driver's 2*nx
% y-period), L (2*pi), K_d2 (f/Cg), shear (0), k_scale (1), nsub (5),
% bump (1e-10, interpolate.m:13 of the QG drivers), device (0).  Returns the packets at the last frame's time.
% The Python twin is swraytracing_amd.trace_stored.
    if nargin < 7, opts = struct(); end
    nlayers = opt(opts, 'nlayers', 1);
    L = opt(opts, 'L', 2*pi);
    K_d2 = opt(opts, 'K_d2', f / Cg);
    shear = opt(opts, 'shear', 0);
    k_scale = opt(opts, 'k_scale', 1);
    nsub = opt(opts, 'nsub', 5);
    bump = opt(opts, 'bump', 1e-10);
    frames = opt(opts, 'frames', []);
    if isempty(frames)
        d = dir([pv_path '.bin']);
        frames = 1:(d.bytes / (8 * nx * nx * nlayers));
    end
    times = opt(opts, 'times', []);
    if isempty(times)
        tall = read_field(fullfile(fileparts(pv_path), 'pv_time'));
        times = tall(frames);
    end
    if numel(frames) < 2 || numel(times) ~= numel(frames) || any(diff(times) <= 0)
        error('swrt:arg', 'need two or more frames with increasing times');
    end
    ctx = SwrtContext(opt(opts, 'device', 0));   % freed when this function returns
    h = ctx.id();
    ny_period = nx * nlayers;
    swrt_mex('packets_set', h, x, k);
    swrt_mex('set_locality', h, 4 * nsub, 0);   % re-binning at interval ends: whole intervals per launch
    load_frame(0, frames(1));
    i = 2;
    while i <= numel(frames)
        g = min(4, numel(frames) - i + 1);
        for j = 0:g-1
            load_frame(1 + j, frames(i + j));
        end
        % per-interval leapfrog step, gH = Cg^2, alpha = (s + 1/2)/nsub
        swrt_mex('advance_intervals', h, diff(times(i-1:i+g-1)) / nsub, nsub, f, Cg^2, 0.5 / nsub, 1 / nsub, bump);
        swrt_mex('swap_slots', h, 0, g);   % the last frame starts the next call
        i = i + g;
    end
    [x, k] = swrt_mex('packets_get', h);
    t_end = times(end);

    function load_frame(slot, fr)
        q = read_field(pv_path, nx, nx, nlayers, fr);
        swrt_mex('set_field_q', h, slot, q(:, :, 1), L, K_d2, shear, k_scale, ny_period);
    end
end

function v = opt(s, name, default)
    if isfield(s, name), v = s.(name); else, v = default; end
end
