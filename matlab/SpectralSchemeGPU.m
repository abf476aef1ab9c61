classdef SpectralSchemeGPU < RaytracingScheme
    % Drop-in for SpectralScheme (SpectralScheme.m:1-70) backed by the MI355X
    % library through swrt_mex: same constructor signature, same U / grad_U
    % / streamfunction results (bit-identical interpolation arithmetic).
    properties
        L, nx, bump, psi_field
    end
    methods
        function obj = SpectralSchemeGPU(L, nx, psi_field)
            swrt_mex('create', 0);
            obj.L = L;
            obj.nx = nx;
            obj.bump = 1e-13;   % ray_trace_sw/interpolate.m (addpath order of the original ctor)
            swrt_mex('set_field_psi', 0, psi_field, L);
            obj.psi_field = swrt_mex('k2g', swrt_mex('g2k', psi_field));   % SpectralScheme.m:28
        end

        function psi = streamfunction(obj, x, y, t)
            dx = obj.L / obj.nx;                                           % SpectralScheme.m:38-43
            psi = reshape(swrt_mex('interpolate', x, y, obj.psi_field, dx, dx, obj.bump), size(x));
        end

        function u = U(obj, x, t)
            xx = x(:,1,:); yy = x(:,2,:);
            I = swrt_mex('eval', xx(:), yy(:), 1, 0, obj.bump);
            u = zeros(size(x));
            u(:,1,:) = reshape(I(:,1), size(xx));
            u(:,2,:) = reshape(I(:,2), size(xx));
        end

        function nablaU = grad_U(obj, x, t)
            xx = x(:,1,:); yy = x(:,2,:);
            I = swrt_mex('eval', xx(:), yy(:), 1, 0, obj.bump);
            nablaU.u_x = I(:,3); nablaU.u_y = I(:,4);
            nablaU.v_x = I(:,5); nablaU.v_y = I(:,6);
        end
    end
end
