classdef SwrtContext < handle
    % One library context (swrt_mex('create')) owned by reference: value
    % objects that hold it (SpectralSchemeGPU, and its copies) share one
    % SwrtContext, and MATLAB calls delete — which destroys the context and
    % frees its device memory (field slots, packets, streams) — when the last
    % reference goes away.  release() closes it early for every holder; a
    % later call through any copy then fails with "closed context".
    properties (SetAccess = private)
        h = 0       % swrt_mex handle; 0 once closed
    end
    methods
        function obj = SwrtContext(device)
            if nargin < 1, device = 0; end
            obj.h = swrt_mex('create', device);
        end

        function h = id(obj)
            if obj.h == 0
                error('swrt:state', 'closed context');
            end
            h = obj.h;
        end

        function release(obj)
            if obj.h ~= 0
                swrt_mex('destroy', obj.h);
                obj.h = 0;
            end
        end

        function delete(obj)
            obj.release();
        end
    end
end
