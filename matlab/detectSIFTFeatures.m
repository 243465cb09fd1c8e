function points = detectSIFTFeatures(I, varargin)
%DETECTSIFTFEATURES libvo (MI355X) shadow of the Computer Vision Toolbox function.
%   points = detectSIFTFeatures(I)            reference call site: VO.m:79-80
%   Only the defaults VO.m uses (ContrastThreshold 0.0133, EdgeThreshold 10,
%   NumLayersInOctave 3, Sigma 1.6) are supported.  Detection and the SIFT
%   descriptors run in one device pass (vo_mex 'sift'); the descriptors are
%   kept for the extractFeatures shadow.  I is handed over in MATLAB's own
%   column-major storage (no host transpose).
    if ~isempty(varargin)
        error('vo:detectSIFTFeatures:options', 'libvo implements the default options only');
    end
    if ~isa(I, 'uint8')
        I = im2uint8(I);
    end
    [loc, scale, ori, metric, desc, octave, layer] = vo_mex('sift', I);
    vo_sift_cache('put', I, loc, desc);
    points = SIFTPoints(loc, 'Scale', scale, 'Orientation', ori, 'Metric', metric, ...
                        'Octave', octave, 'Layer', layer);
end
