/*
 * HipMODWTTransform — MODWTTransform.forwardMODWT / inverseMODWT
 * (MODWTTransform.java:256-375, DIRECT semantics) on libjwave_hip.so.
 * The flattened pow-2 API (:389-443) is inherited and calls these.
 */
package jwave.amd;

import jwave.exceptions.JWaveException;
import jwave.transforms.MODWTTransform;
import jwave.transforms.wavelets.Wavelet;

public class HipMODWTTransform extends MODWTTransform {

  private final HipNative.Taps _taps;

  public HipMODWTTransform( Wavelet wavelet ) {
    super( wavelet );
    _taps = HipNative.tapsFor( wavelet );
  }

  @Override public double[ ][ ] forwardMODWT( double[ ] data, int maxLevel ) {
    if( _taps == null || data == null || data.length == 0 )
      return super.forwardMODWT( data, maxLevel ); // reference checks + empty rows
    int n = data.length;
    if( maxLevel < 0 || !HipNative.fitsArray( maxLevel + 1, n ) )
      return super.forwardMODWT( data, maxLevel );  // reference checks, or > one Java array
    double[ ] wv = new double[ ( maxLevel + 1 ) * n ];
    try {
      HipNative.check( HipNative.modwt( HipNative.ctx( ), true, data, wv, n, maxLevel, _taps.L,
          _taps.tw, _taps.lo, _taps.hi, _taps.loR, _taps.hiR ) );
    } catch( JWaveException e ) {
      throw new IllegalStateException( e.getMessage( ), e );
    }
    return HipNative.unpack( wv, maxLevel + 1, n );
  }

  @Override public double[ ] inverseMODWT( double[ ][ ] c ) {
    if( _taps == null || c == null || c.length <= 1 )
      return super.inverseMODWT( c );
    int J = c.length - 1, n = c[ 0 ].length;
    if( !HipNative.fitsArray( J + 1, n ) )
      return super.inverseMODWT( c );
    double[ ] wv = HipNative.pack( c ), x = new double[ n ];
    try {
      HipNative.check( HipNative.modwt( HipNative.ctx( ), false, x, wv, n, J, _taps.L, _taps.tw,
          _taps.lo, _taps.hi, _taps.loR, _taps.hiR ) );
    } catch( JWaveException e ) {
      throw new IllegalStateException( e.getMessage( ), e );
    }
    return x;
  }

  /**
   * forwardMODWT of every signal (equal lengths), in one native call that
   * spreads contiguous blocks of signals over the -Djwave.hip.devices GPUs
   * (else this thread's device).  Each result is forwardMODWT(signals[i],
   * maxLevel) bit for bit; the reference's checks (empty input, levels) run
   * per signal through the single-signal path.
   */
  public double[ ][ ][ ] forwardMODWT( double[ ][ ] signals, int maxLevel ) {
    int b = signals.length, n = b == 0 ? 0 : signals[ 0 ].length;
    boolean native_ = _taps != null && b > 0 && n > 0 && maxLevel >= 0
        && HipNative.fitsArray( (long)b * ( maxLevel + 1 ), n );
    for( int i = 0; native_ && i < b; i++ )
      native_ = signals[ i ] != null && signals[ i ].length == n;
    if( !native_ ) {
      double[ ][ ][ ] out = new double[ b ][ ][ ];
      for( int i = 0; i < b; i++ )
        out[ i ] = forwardMODWT( signals[ i ], maxLevel );
      return out;
    }
    try {
      return HipNative.modwtForwardBatch( _taps, signals, maxLevel );
    } catch( JWaveException e ) {
      throw new IllegalStateException( e.getMessage( ), e );
    }
  }

  /** inverseMODWT of every signal's coefficients (equal shapes), one native call. */
  public double[ ][ ] inverseMODWT( double[ ][ ][ ] coefficients ) {
    int b = coefficients.length;
    boolean native_ = _taps != null && b > 0 && coefficients[ 0 ] != null
        && coefficients[ 0 ].length > 1;
    int J = native_ ? coefficients[ 0 ].length - 1 : 0;
    int n = native_ ? coefficients[ 0 ][ 0 ].length : 0;
    native_ = native_ && n > 0 && HipNative.fitsArray( (long)b * ( J + 1 ), n );
    for( int i = 0; native_ && i < b; i++ ) {
      native_ = coefficients[ i ] != null && coefficients[ i ].length == J + 1;
      for( int r = 0; native_ && r <= J; r++ )
        native_ = coefficients[ i ][ r ] != null && coefficients[ i ][ r ].length == n;
    }
    if( !native_ ) {
      double[ ][ ] out = new double[ b ][ ];
      for( int i = 0; i < b; i++ )
        out[ i ] = inverseMODWT( coefficients[ i ] );
      return out;
    }
    try {
      return HipNative.modwtInverseBatch( _taps, coefficients );
    } catch( JWaveException e ) {
      throw new IllegalStateException( e.getMessage( ), e );
    }
  }
}
