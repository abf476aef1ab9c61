function [x, k, t] = ode_symplectic_gpu(x0, k0, dt, T, f, gH, scheme)
% Drop-in for ode_symplectic (ode_symplectic.m:1-31): same arguments, same
% Nsteps x 2 x P outputs.  With a SpectralSchemeGPU the whole time loop is one
% fused device pass (swrt_leapfrog); any other scheme falls back to the
% reference implementation.
    if ~isa(scheme, 'SpectralSchemeGPU')
        [x, k, t] = ode_symplectic(x0, k0, dt, T, f, gH, scheme);
        return
    end
    Nsteps = floor(T / dt);
    P = size(x0, 3);
    x = zeros([Nsteps, 2, P]);
    k = zeros([Nsteps, 2, P]);
    t = (0:Nsteps-1)' * dt;
    x(1, :, :) = x0;
    k(1, :, :) = k0;
    if Nsteps < 2
        return
    end
    X0 = reshape(x0, 2, P)';   % P x 2 (packet_x layout)
    K0 = reshape(k0, 2, P)';
    [~, ~, hx, hk] = swrt_mex('leapfrog', scheme.h, X0, K0, dt, Nsteps - 1, f, gH, 1, 0, 0, scheme.bump, 1);
    % hx: P x 2 x (Nsteps-1) frames -> Nsteps x 2 x P
    x(2:end, :, :) = permute(hx, [3 2 1]);
    k(2:end, :, :) = permute(hk, [3 2 1]);
end
