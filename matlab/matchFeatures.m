function indexPairs = matchFeatures(features1, features2, varargin)
%MATCHFEATURES libvo (MI355X) shadow: indexPairs = matchFeatures(features1, features2)
%   reference call sites: VO.m:87,283,293,311,323.  Defaults only (Exhaustive,
%   SSD, MatchThreshold 1.0, MaxRatio 0.6, Unique false).  The N x 128 single
%   descriptors are handed over as they lie (column-major, no conversion on
%   the host); indexPairs is P x 2 uint32, ascending in the first column.
%   u8-valued rows (extractFeatures' SIFT descriptors, all VO.m passes) take
%   libvo's exact-integer path; any other single features take its float SSD
%   path (rows normalised to unit length, SSD summed in a fixed order).
    if ~isempty(varargin) || nargout > 1
        error('vo:matchFeatures:options', 'libvo implements indexPairs = matchFeatures(F1, F2) with the default options');
    end
    indexPairs = vo_mex('match', single(features1), single(features2));
end
