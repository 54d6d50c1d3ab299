package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.cluster.TokenResult;
import com.alibaba.csp.sentinel.cluster.TokenResultStatus;
import com.alibaba.csp.sentinel.cluster.TokenService;
import com.alibaba.csp.sentinel.cluster.flow.DefaultTokenService;
import com.alibaba.csp.sentinel.spi.Spi;

import java.util.Collection;

/**
 * Drop-in TokenService for sentinel-cluster-server-default: TokenServiceProvider
 * resolves with loadFirstInstanceOrDefault and DefaultTokenService is the
 * default (DefaultTokenService.java:35), so this provider wins when listed in
 * META-INF/services.  requestToken / requestParamToken are batched into
 * sf_request_tokens (ClusterFlowChecker / ClusterParamFlowChecker on the GPU);
 * the argument checks are the reference's (DefaultTokenService.java:40-62).
 * Concurrent tokens stay on the reference implementation.
 */
@Spi(order = -100)
public final class GpuTokenService implements TokenService {
    private static final TokenService DEFAULT = new DefaultTokenService();
    private final TokenBatcher batcher = TokenBatcher.get();

    @Override
    public TokenResult requestToken(Long ruleId, int acquireCount, boolean prioritized) {
        if (ruleId == null || ruleId <= 0 || acquireCount <= 0) return new TokenResult(TokenResultStatus.BAD_REQUEST);
        return batcher.request(ruleId, acquireCount, prioritized, null);
    }

    @Override
    public TokenResult requestParamToken(Long ruleId, int acquireCount, Collection<Object> params) {
        if (ruleId == null || ruleId <= 0 || acquireCount <= 0 || params == null || params.isEmpty()) {
            return new TokenResult(TokenResultStatus.BAD_REQUEST);
        }
        return batcher.request(ruleId, acquireCount, false, params.toArray());
    }

    @Override
    public TokenResult requestConcurrentToken(String clientAddress, Long ruleId, int acquireCount) {
        return DEFAULT.requestConcurrentToken(clientAddress, ruleId, acquireCount);
    }

    @Override
    public void releaseConcurrentToken(Long tokenId) {
        DEFAULT.releaseConcurrentToken(tokenId);
    }
}
