function [worldPose, inlierIdx, status] = estworldpose(imagePoints, worldPoints, intrinsics, varargin)
%ESTWORLDPOSE libvo (MI355X) shadow: P3P + MSAC camera pose in the world frame.
%   [worldPose, inlierIdx, status] = estworldpose(imagePoints, worldPoints, intrinsics, ...
%       'MaxNumTrials', 1000, 'Confidence', 99, 'MaxReprojectionError', 1)
%   reference call site: VO.m:123-127 (defaults).  Without the status output a
%   failure throws, as the toolbox function does; with it, status is 1 (not
%   enough points) or 2 (not enough inliers) and worldPose is the identity.
%   MaxNumTrials is limited to the context's 1000 hypothesis slots.
    p = inputParser;
    p.addParameter('MaxNumTrials', 1000);
    p.addParameter('Confidence', 99);
    p.addParameter('MaxReprojectionError', 1);
    p.parse(varargin{:});
    opts = double([p.Results.MaxNumTrials, p.Results.Confidence, p.Results.MaxReprojectionError]);
    if nargout > 2
        [A, inlierIdx, status] = vo_mex('estworldpose', double(imagePoints), double(worldPoints), double(intrinsics.K), opts);
    else
        [A, inlierIdx] = vo_mex('estworldpose', double(imagePoints), double(worldPoints), double(intrinsics.K), opts);
    end
    worldPose = rigidtform3d(A);
end
