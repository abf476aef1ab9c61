classdef SpectralSchemeGPU < RaytracingScheme
    % Drop-in for SpectralScheme (SpectralScheme.m:1-70) backed by the MI355X
    % library through swrt_mex: same constructor signature, same properties
    % (U_field, GradU_field, psi_field, L; SpectralScheme.m:3) and the same
    % U / grad_U / streamfunction results (bit-identical interpolation
    % arithmetic on the device's fields).  Each instance holds a library
    % context with its fields, as each SpectralScheme owns its fields
    % (SpectralScheme.m:28-35).  The context is a SwrtContext (a handle
    % object): copies of a scheme share it and it is destroyed with its last
    % reference, so building one scheme per snapshot does not accumulate
    % device memory; release(scheme) frees it early for every copy.
    properties
        L, nx, bump, psi_field, ctx
    end
    properties (Dependent)
        h                       % the swrt_mex handle of ctx (errors once released)
        U_field, GradU_field    % downloaded from the device on access
    end
    methods
        function obj = SpectralSchemeGPU(L, nx, psi_field)
            obj.ctx = SwrtContext(0);
            obj.L = L;
            obj.nx = nx;
            obj.bump = 1e-13;   % ray_trace_sw/interpolate.m (addpath order of the original ctor)
            swrt_mex('set_field_psi', obj.h, 0, psi_field, L);
            obj.psi_field = swrt_mex('get_psi', obj.h, 0, nx);        % k2g(g2k(psi)), SpectralScheme.m:28
        end

        function s = get.U_field(obj)                                  % SpectralScheme.m:29-30
            F = swrt_mex('get_fields', obj.h, 0, obj.nx);
            s.u = F(:,:,1); s.v = F(:,:,2);
        end

        function s = get.GradU_field(obj)                              % SpectralScheme.m:32-35
            F = swrt_mex('get_fields', obj.h, 0, obj.nx);
            s.u_x = F(:,:,3); s.u_y = F(:,:,4); s.v_x = F(:,:,5); s.v_y = F(:,:,6);
        end

        function h = get.h(obj)
            h = obj.ctx.id();
        end

        function release(obj)
            obj.ctx.release();
        end

        function psi = streamfunction(obj, x, y, t)
            dx = obj.L / obj.nx;                                       % SpectralScheme.m:38-43
            psi = reshape(swrt_mex('interpolate', obj.h, x, y, obj.psi_field, dx, dx, obj.bump), size(x));
        end

        function u = U(obj, x, t)
            xx = x(:,1,:); yy = x(:,2,:);
            I = swrt_mex('eval', obj.h, xx(:), yy(:), 1, 0, obj.bump);
            u = zeros(size(x));
            u(:,1,:) = reshape(I(:,1), size(xx));
            u(:,2,:) = reshape(I(:,2), size(xx));
        end

        function nablaU = grad_U(obj, x, t)
            xx = x(:,1,:); yy = x(:,2,:);
            I = swrt_mex('eval', obj.h, xx(:), yy(:), 1, 0, obj.bump);
            nablaU.u_x = I(:,3); nablaU.u_y = I(:,4);
            nablaU.v_x = I(:,5); nablaU.v_y = I(:,6);
        end
    end
end
