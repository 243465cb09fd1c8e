function [features, validPoints] = extractFeatures(I, points, varargin)
%EXTRACTFEATURES libvo (MI355X) shadow for extractFeatures(I, points, "Method", "SIFT").
%   [features, validPoints] = extractFeatures(I, points, "Method", "SIFT")
%   reference call site: VO.m:83-84.  Returns the N x 128 single descriptors
%   the detectSIFTFeatures shadow computed for these points of this image in
%   the same device pass; every point gets a descriptor (validPoints = points).
    if numel(varargin) ~= 2 || ~strcmpi(string(varargin{1}), "Method") || ~strcmpi(string(varargin{2}), "SIFT")
        error('vo:extractFeatures:options', 'libvo implements extractFeatures(I, points, "Method", "SIFT") only');
    end
    if ~isa(I, 'uint8')
        I = im2uint8(I);
    end
    desc = vo_sift_cache('get', I, points.Location);
    if isempty(desc)                       % not the last detections of this image: detect again
        [loc, ~, ~, ~, desc] = vo_mex('sift', I);
        if ~isequal(loc, points.Location)
            error('vo:extractFeatures:points', 'libvo describes the points its own detectSIFTFeatures returned');
        end
    end
    features = desc;
    validPoints = points;
end
